"""Device training engine: the hot path of ``submodel_trainer.py`` on MI355X.

What the reference does per step (``submodel_trainer.py:250-302``, model and
optimizer from ``:606-660``), and where it runs here:

* front end of ``SpectrogramDataset.__getitem__`` (``:189-208``) -- mel
  (norm=None, quirk C3) + dB: ``FrontEnd(norm=None)``; SpecAugment masks +
  standardise: ``sad_specaug_norm_run``; Resize(512) + RandomResizedCrop:
  ``sad_crop_resize_run`` (``TrainFrontEnd``).
* ``outputs = model(inputs)`` with ``model.train()``: timm ResNet-18 with
  batch-statistics BatchNorm (running stats updated, momentum 0.1) and global
  average pooling -> pooled features ``[B, 512]`` (the attached head is never
  called, quirk C1): ``TrainNet.forward_train`` -- raw MFMA convs
  (``sad_conv2d_run``, ``sad_stem_conv_run``), ``sad_bn_stats_run``,
  ``sad_bn_apply_run`` / ``sad_bn_relu_maxpool_run``, ``sad_avgpool_run``.
* ``CrossEntropyLoss`` on those 512 "logits": ``sad_ce_loss_run``.
* ``loss.backward()`` into the trainable stages (layer4; layer3 once unfrozen,
  quirk C4): ``TrainNet.backward`` -- ``sad_bn_backward_run``, dgrad as an
  MFMA conv over flipped weights (stride 1) or GEMM + col2im (stride 2),
  wgrad as im2col + GEMM (``sad_conv_wgrad_run``).
* ``clip_grad_norm_(0.5)`` + ``AdamW(lr, wd=0.01)``: ``sad_clip_grad_norm_run``,
  ``sad_adamw_run`` over flat fp32 buffers.
* ``DataParallel`` -> one process per GPU (``torch.distributed`` over RCCL):
  per-replica BN statistics as in DP, one all-reduce (SUM) of the step's
  trainable gradients per step; the loss is scaled by 1 / global batch so the
  sum equals DP's gradient of the global-batch mean.

Master weights, BN statistics, gradients and optimizer moments are fp32;
activations are bf16 (throughput) or fp32 (parity) NHWC.
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import Dict, List

import numpy as np
import torch

from . import _lib
from .engine import MAP_H, MAP_W, Backbone, FrontEnd, ResNetBackbone, _dev
from .weights import HEAD_LAYOUT, arch_param_shapes, arch_spec, backbone_param_shapes, head_layout

BN_EPS = 1e-5
BN_MOMENTUM = 0.1
IMG = 512
FEATURES = 512
ADAM_BETAS = (0.9, 0.999)
ADAM_EPS = 1e-8
WEIGHT_DECAY = 0.01
MAX_GRAD_NORM = 0.5


def block_table(layers=(2, 2, 2, 2)):
    """[(prefix, cin, cout, stride, has_downsample)] of a timm BasicBlock ResNet
    (resnet18 by default; resnet34 = (3, 4, 6, 3))."""
    out, inp = [], 64
    for li, planes in enumerate((64, 128, 256, 512)):
        for b in range(layers[li]):
            s = 2 if (b == 0 and li > 0) else 1
            out.append((f'layer{li + 1}.{b}', inp, planes, s, b == 0 and li > 0))
            inp = planes
    return out


BLOCKS = block_table()


def bottleneck_table(layers=(3, 4, 6, 3)):
    """[(prefix, cin, cout, stride, has_downsample, width)] of a timm Bottleneck
    ResNet (resnet50/101/152): width = planes, cout = 4 * planes, stride on conv2,
    a downsample wherever the shape changes (incl. layer1.0: 64 -> 256)."""
    out, inp = [], 64
    for li, planes in enumerate((64, 128, 256, 512)):
        for b in range(layers[li]):
            s = 2 if (b == 0 and li > 0) else 1
            out.append((f'layer{li + 1}.{b}', inp, 4 * planes, s, b == 0, planes))
            inp = 4 * planes
    return out


def _blocks(model_name: str):
    """(is_bottleneck, block table, num_features) of a supported timm ResNet."""
    block, layers, nf = arch_spec(model_name)
    if block == 'bottleneck':
        return True, bottleneck_table(layers), nf
    return False, block_table(layers), nf


def param_layout(model_name: str = 'resnet18'):
    """[(name, shape)] of the backbone's parameters in timm ``parameters()`` order."""
    out = []
    for key, shape, kind in arch_param_shapes(model_name):
        if kind == 'conv':
            out.append((f'{key}.weight', shape))
        else:
            out.append((f'{key}.weight', shape))
            out.append((f'{key}.bias', shape))
    return out


def head_keys():
    """state-dict keys of the trainer's ``model.head`` (``submodel_trainer.py:613-625``)."""
    keys = []
    for idx, kind, _ in HEAD_LAYOUT:
        keys += [f'{idx}.weight', f'{idx}.bias']
        if kind == 'bn':
            keys += [f'{idx}.running_mean', f'{idx}.running_var', f'{idx}.num_batches_tracked']
    return keys


# BinaryClassifier head in train mode (--head-loss): Dropout rates of the
# reference's model.head (submodel_trainer.py:613-625)
HEAD_DROPOUT = (0.5, 0.3)


def head_param_layout(num_features: int = 512):
    """[(name, shape)] of model.head's parameters in ``parameters()`` order
    (nn.Sequential indices 2, 3, 6, 7, 10): the layout of
    sad_head_train_backward_run's gradient buffer."""
    out = []
    for idx, kind, shape in head_layout(num_features):
        out += [(f'head.{idx}.weight', shape), (f'head.{idx}.bias', (shape[0],))]
    return out


# --------------------------------------------------------------- initialisation
def init_state_dict(seed: int = 42, model_name: str = 'resnet18'):
    """Initial trainer model, ``torch.manual_seed(seed)`` then
    ``timm.create_model('resnet18', pretrained=False, num_classes=0)`` and the
    MLP head (``submodel_trainer.py:599-625``), reproduced by making the same CPU
    RNG draws in the same order: every Conv2d/Linear's construction-time
    ``reset_parameters`` (timm builds a stage's downsample before its blocks),
    then timm's ``init_weights`` (kaiming_normal_ fan_out / relu on every conv in
    module order, BN 1/0, ``zero_init_last``: every BasicBlock's bn2.weight = 0).
    timm is not installed here, so bit-identity with it is unpinned.
    Returns (backbone_sd, head_sd) with timm / nn.Sequential keys."""
    g = torch.Generator().manual_seed(seed)
    layout = arch_param_shapes(model_name)
    convs = {k: torch.empty(s) for k, s, kind in layout if kind == 'conv'}
    # construction order: conv1, then per stage: downsample.0, block convs
    order = ['conv1']
    bottleneck, blocks, nf = _blocks(model_name)
    for prefix, _, _, _, has_ds, *_ in blocks:
        if has_ds:
            order.append(f'{prefix}.downsample.0')
        order += [f'{prefix}.conv1', f'{prefix}.conv2'] + ([f'{prefix}.conv3'] if bottleneck else [])
    for k in order:
        torch.nn.init.kaiming_uniform_(convs[k], a=math.sqrt(5), generator=g)
    sd = OrderedDict()
    for k, s, kind in layout:  # named_modules order == state-dict order
        if kind == 'conv':
            torch.nn.init.kaiming_normal_(convs[k], mode='fan_out', nonlinearity='relu', generator=g)
            sd[f'{k}.weight'] = convs[k]
        else:
            c = s[0]
            last = '.bn3' if bottleneck else '.bn2'  # zero_init_last
            w = torch.zeros(c) if k.endswith(last) else torch.ones(c)
            sd[f'{k}.weight'], sd[f'{k}.bias'] = w, torch.zeros(c)
            sd[f'{k}.running_mean'], sd[f'{k}.running_var'] = torch.zeros(c), torch.ones(c)
            sd[f'{k}.num_batches_tracked'] = torch.tensor(0, dtype=torch.long)
    hd = OrderedDict()
    for idx, kind, shape in head_layout(nf):
        if kind == 'linear':  # nn.Linear.reset_parameters
            w = torch.empty(shape)
            torch.nn.init.kaiming_uniform_(w, a=math.sqrt(5), generator=g)
            bound = 1.0 / math.sqrt(shape[1])
            b = torch.empty(shape[0]).uniform_(-bound, bound, generator=g)
            hd[f'{idx}.weight'], hd[f'{idx}.bias'] = w, b
        else:
            c = shape[0]
            hd[f'{idx}.weight'], hd[f'{idx}.bias'] = torch.ones(c), torch.zeros(c)
            hd[f'{idx}.running_mean'], hd[f'{idx}.running_var'] = torch.zeros(c), torch.ones(c)
            hd[f'{idx}.num_batches_tracked'] = torch.tensor(0, dtype=torch.long)
    return sd, hd


# ------------------------------------------------------------------- front end
class TrainFrontEnd:
    """SpectrogramDataset's per-segment transform chain on the device
    (``submodel_trainer.py:97-114,189-206,463-471``): waveform [n, 128000]
    fp32 -> image [n, 512, 512] (one of the three identical channels)."""

    def __init__(self, device='cuda', dtype: str = 'bf16'):
        self.device = _dev(device)
        self.fe = FrontEnd(self.device, norm=None, top_db=80.0)
        self.dtype = dtype
        self._dt = _lib.SAD_BF16 if dtype == 'bf16' else _lib.SAD_F32
        self.tdtype = torch.bfloat16 if dtype == 'bf16' else torch.float32

    def maps(self, wave: torch.Tensor, masks: torch.Tensor | None = None) -> torch.Tensor:
        """standardised maps [n, 128, 251]; masks int32 [n, 4] (f0, f1, t0, t1) or None."""
        m, db = self.fe(wave, want_db=True)
        if masks is None:
            return m
        masks = masks.to(self.device, torch.int32).contiguous()
        out = torch.empty_like(m)
        with torch.cuda.device(self.device):
            _lib.call('sad_specaug_norm_run', _lib.ptr(db), m.shape[0], MAP_H, MAP_W, _lib.ptr(masks), _lib.ptr(out),
                      _lib.stream_handle(self.device))
        return out

    def images(self, maps: torch.Tensor, boxes: torch.Tensor | None = None) -> torch.Tensor:
        """[n, 512, 512] in the compute dtype; boxes int32 [n, 4] (i, j, h, w) or None."""
        n = maps.shape[0]
        img = torch.empty(n, IMG, IMG, device=self.device, dtype=self.tdtype)
        if boxes is not None:
            boxes = boxes.to(self.device, torch.int32).contiguous()
        with torch.cuda.device(self.device):
            _lib.call('sad_crop_resize_run', _lib.ptr(maps), n, MAP_H, MAP_W, _lib.ptr(boxes), IMG, self._dt,
                      _lib.ptr(img), _lib.stream_handle(self.device))
        return img

    def __call__(self, wave, masks=None, boxes=None):
        return self.images(self.maps(wave, masks), boxes)


# ------------------------------------------------------------------- network
class TrainNet:
    """timm resnet18 / resnet34 (+ the unused MLP head) in train mode on one device."""

    def __init__(self, base_sd: Dict[str, torch.Tensor], head_sd: Dict[str, torch.Tensor], device='cuda',
                 dtype: str = 'bf16', model_name: str = 'resnet18', head_loss: bool = False):
        self.device = _dev(device)
        self.model_name = model_name
        self.bottleneck, self.blocks, self.num_features = _blocks(model_name)
        self.dtype = dtype
        self._dt = _lib.SAD_BF16 if dtype == 'bf16' else _lib.SAD_F32
        self.tdtype = torch.bfloat16 if dtype == 'bf16' else torch.float32
        self.es = 2 if dtype == 'bf16' else 4
        layout = param_layout(model_name)
        # --head-loss: the head's parameters follow the backbone's in the flat
        # buffers (parameters() order), so the layer4 range's all-reduce, clip
        # and AdamW cover them as the reference's optimizer does (:648-652)
        self.head_loss = head_loss
        if head_loss:
            layout = layout + head_param_layout(self.num_features)
        self.names = [n for n, _ in layout]
        sizes = [int(np.prod(s)) for _, s in layout]
        offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        self.offsets = {n: (int(offs[i]), int(offs[i + 1])) for i, n in enumerate(self.names)}
        total = int(offs[-1])
        self.pflat = torch.empty(total, device=self.device, dtype=torch.float32)
        self.gflat = torch.zeros(total, device=self.device, dtype=torch.float32)
        self.params, self.grads = OrderedDict(), OrderedDict()
        for (n, s), (a, b) in zip(layout, [self.offsets[n] for n in self.names]):
            self.params[n] = self.pflat[a:b].view(s)
            self.grads[n] = self.gflat[a:b].view(s)
            src = head_sd[n[5:]] if n.startswith('head.') else base_sd[n]
            self.params[n].copy_(torch.as_tensor(src, dtype=torch.float32))
        self.bn_keys = [k for k, _, kind in arch_param_shapes(model_name) if kind == 'bn']
        self.running = {}
        self.nbt = {}
        for k in self.bn_keys:
            self.running[k] = (torch.as_tensor(base_sd[f'{k}.running_mean'], dtype=torch.float32).to(self.device).clone(),
                               torch.as_tensor(base_sd[f'{k}.running_var'], dtype=torch.float32).to(self.device).clone())
            self.nbt[k] = int(torch.as_tensor(base_sd.get(f'{k}.num_batches_tracked', 0)).item())
        self.head_sd = OrderedDict((k, torch.as_tensor(head_sd[k]).detach().clone().cpu()) for k in head_keys())
        if head_loss:  # the head's BN running statistics live on the device while it trains
            self.head_running = {i: tuple(torch.as_tensor(head_sd[f'{i}.{b}'], dtype=torch.float32).to(self.device)
                                          .clone() for b in ('running_mean', 'running_var')) for i in (3, 7)}
            self.head_nbt = {i: int(torch.as_tensor(head_sd.get(f'{i}.num_batches_tracked', 0)).item())
                             for i in (3, 7)}
            self.range_head = self.offsets['head.2.weight'][0], total
        self.range4 = (self.offsets['layer4.0.conv1.weight'][0], total)
        self.range3 = (self.offsets['layer3.0.conv1.weight'][0], self.range4[0])
        self.zero_bias = torch.zeros(max(FEATURES, self.num_features), device=self.device, dtype=torch.float32)
        self._packed = {}
        self._ws = {}
        self.update_running = True

    # ---------------------------------------------------------- utilities
    def _stream(self):
        return _lib.stream_handle(self.device)

    def _buf(self, name: str, nbytes: int) -> torch.Tensor:
        b = self._ws.get(name)
        if b is None or b.numel() < nbytes:
            b = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=self.device)
            self._ws[name] = b
        return b

    def packed(self, conv: str, mode: int) -> torch.Tensor:
        """Compute-dtype copy of conv weight ``conv`` in pack ``mode`` (cached
        until the weight changes)."""
        key = (conv, mode)
        t = self._packed.get(key)
        if t is None:
            w = self.params[f'{conv}.weight']
            co, ci, k, _ = w.shape
            n = co * 64 if mode in (2, 4) else w.numel()
            t = torch.empty(n, device=self.device, dtype=self.tdtype)
            with torch.cuda.device(self.device):
                _lib.call('sad_pack_conv_weight_run', _lib.ptr(w), co, ci, k, mode, self._dt, _lib.ptr(t),
                          self._stream())
            self._packed[key] = t
        return t

    def invalidate_packed(self):
        """Drop every cached weight pack (after the parameters were overwritten)."""
        self._packed.clear()

    def invalidate(self, prefix: str, keep_modes=()):
        for key in [k for k in self._packed if k[0].startswith(prefix) and k[1] not in keep_modes]:
            del self._packed[key]

    def pack_segments(self, prefix: str, base: int):
        """sad_pack_seg entries for the conv weights under ``prefix`` whose
        pack-mode 0 / 1 copies are cached (offsets relative to flat index
        ``base``), for sad_adamw_pack_run."""
        segs = []
        for name in self.names:
            if not (name.startswith(prefix) and name.endswith('.weight')):
                continue
            conv = name[:-len('.weight')]
            m0, m1 = self._packed.get((conv, 0)), self._packed.get((conv, 1))
            w = self.params[name]
            if w.dim() != 4 or (m0 is None and m1 is None):
                continue
            co, ci, k, _ = w.shape
            segs.append(_lib.PackSeg(self.offsets[name][0] - base, co, ci, k, 0, _lib.ptr(m0), _lib.ptr(m1)))
        assert len(segs) <= 16
        return segs

    def _bn_stats(self, x: torch.Tensor, key: str) -> torch.Tensor:
        C = x.shape[-1]
        P = x.numel() // C
        st = torch.empty(4 * C, device=self.device, dtype=torch.float32)
        sz = _lib.SZ()
        _lib.call('sad_bn_workspace_size', P, C, _lib.ctypes.byref(sz))
        ws = self._buf('bn', sz.value)
        rm, rv = self.running[key] if self.update_running else (None, None)
        with torch.cuda.device(self.device):
            _lib.call('sad_bn_stats_run', _lib.ptr(x), P, C, self._dt, _lib.ptr(self.params[f'{key}.weight']),
                      _lib.ptr(self.params[f'{key}.bias']), BN_EPS, BN_MOMENTUM, _lib.ptr(rm), _lib.ptr(rv),
                      _lib.ptr(st), _lib.ptr(ws), ws.numel(), self._stream())
        if self.update_running:
            self.nbt[key] += 1
        return st

    def _conv_bn(self, x, w, cout, k, stride, pad, key):
        """raw conv (pack-mode-0 weights) + its train-mode BN statistics in one
        call (bf16: summed in the conv epilogue)."""
        N, H, W, Cin = x.shape
        Ho, Wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
        out = torch.empty(N, Ho, Wo, cout, device=self.device, dtype=self.tdtype)
        st = torch.empty(4 * cout, device=self.device, dtype=torch.float32)
        sz = _lib.SZ()
        _lib.call('sad_conv_bn_train_workspace_size', N, H, W, cout, k, stride, pad, _lib.ctypes.byref(sz))
        ws = self._buf('convbn', sz.value)
        rm, rv = self.running[key] if self.update_running else (None, None)
        with torch.cuda.device(self.device):
            _lib.call('sad_conv_bn_train_run', _lib.ptr(x), N, H, W, Cin, _lib.ptr(w), cout, k, stride, pad, self._dt,
                      _lib.ptr(self.params[f'{key}.weight']), _lib.ptr(self.params[f'{key}.bias']), BN_EPS,
                      BN_MOMENTUM, _lib.ptr(rm), _lib.ptr(rv), _lib.ptr(st), _lib.ptr(out), _lib.ptr(ws), ws.numel(),
                      None, self._stream())
        if self.update_running:
            self.nbt[key] += 1
        return out, st

    def _bn_apply(self, x, st, res=None, rst=None, relu=True):
        C = x.shape[-1]
        out = torch.empty_like(x)
        with torch.cuda.device(self.device):
            _lib.call('sad_bn_apply_run', _lib.ptr(x), x.numel() // C, C, self._dt, _lib.ptr(st), _lib.ptr(res),
                      _lib.ptr(rst), int(relu), _lib.ptr(out), self._stream())
        return out

    def _conv(self, x, w, cout, k, stride, pad, res=None):
        """raw NHWC conv (no BN) on the MFMA block-conv kernels (the inference
        backbone's); w packed [cout][k][k][cin].  ``res`` (added in the epilogue)
        needs the bf16 halo kernel; fp32 with ``res`` runs the implicit-GEMM kernel."""
        N, H, W, Cin = x.shape
        Ho, Wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
        out = torch.empty(N, Ho, Wo, cout, device=self.device, dtype=self.tdtype)
        with torch.cuda.device(self.device):
            if res is not None and self._dt != _lib.SAD_BF16:
                _lib.call('sad_conv2d_run', _lib.ptr(x), N, H, W, Cin, _lib.ptr(w), _lib.ptr(self.zero_bias),
                          _lib.ptr(res), _lib.ptr(out), cout, k, stride, pad, 0, self._dt, 0, self._stream())
            else:
                _lib.call('sad_block_conv_run', _lib.ptr(x), N, H, W, Cin, None, 0, 0, 0, 1, _lib.ptr(w), 0,
                          _lib.ptr(self.zero_bias), _lib.ptr(res), _lib.ptr(out), cout, k, stride, pad, 0, self._dt,
                          0, self._stream())
        return out

    def _bn_backward(self, x, st, key, grads, dy=None, dpool=None, pool_hw=0, y=None, accumulate=False,
                     want_dz=False):
        C = x.shape[-1]
        P = x.numel() // C
        sz = _lib.SZ()
        _lib.call('sad_bn_workspace_size', P, C, _lib.ctypes.byref(sz))
        ws = self._buf('bn', sz.value)
        dz = torch.empty_like(x) if want_dz else None
        dx = torch.empty_like(x)
        with torch.cuda.device(self.device):
            _lib.call('sad_bn_backward_run', _lib.ptr(x), P, C, self._dt, _lib.ptr(st),
                      _lib.ptr(self.params[f'{key}.weight']), _lib.ptr(dy), _lib.ptr(dpool), pool_hw, _lib.ptr(y),
                      _lib.ptr(grads[f'{key}.weight']), _lib.ptr(grads[f'{key}.bias']), int(accumulate),
                      _lib.ptr(dz), _lib.ptr(dx), _lib.ptr(ws), ws.numel(), self._stream())
        return dx, dz

    def _wgrad(self, x, dy, key, grads, k, stride, pad, beta=0.0):
        N, H, W, Cin = x.shape
        cout = dy.shape[-1]
        sz = _lib.SZ()
        _lib.call('sad_conv_wgrad_workspace_size', N, H, W, Cin, cout, k, stride, pad, self._dt, _lib.ctypes.byref(sz))
        ws = self._buf('wgrad', sz.value)
        with torch.cuda.device(self.device):
            _lib.call('sad_conv_wgrad_run', _lib.ptr(x), N, H, W, Cin, _lib.ptr(dy), cout, k, stride, pad, self._dt,
                      float(beta), _lib.ptr(grads[f'{key}.weight']), _lib.ptr(ws), ws.numel(), self._stream())

    def _dgrad_gemm(self, dy, conv, x_shape, k, stride, pad, dx, accumulate):
        N, Ho, Wo, cout = dy.shape
        _, H, W, Cin = x_shape
        sz = _lib.SZ()
        _lib.call('sad_conv_dgrad_workspace_size', N, Ho, Wo, cout, Cin, k, self._dt, _lib.ctypes.byref(sz))
        ws = self._buf('dgrad', sz.value)
        w = self.packed(conv, 3)
        with torch.cuda.device(self.device):
            _lib.call('sad_conv_dgrad_run', _lib.ptr(dy), N, Ho, Wo, cout, _lib.ptr(w), Cin, H, W, k, stride, pad,
                      self._dt, int(accumulate), _lib.ptr(dx), _lib.ptr(ws), ws.numel(), self._stream())

    # ---------------------------------------------------------- forward
    def forward_train(self, img: torch.Tensor, keep_from: int = 4, stem_chunk: int = 16):
        """img [B, 512, 512] (compute dtype) -> (pooled features [B, 512] fp32,
        saved activations of the blocks of layer >= keep_from)."""
        saved = {}
        a = self.stem_fwd(img, stem_chunk)
        a = self.blocks_fwd(a, self.blocks, saved, keep_from)
        return self.pool(a), saved

    def stem_fwd(self, img: torch.Tensor, stem_chunk: int = 16) -> torch.Tensor:
        """conv1 -> bn1 (batch statistics) -> ReLU -> maxpool: [B, 128, 128, 64]."""
        assert img.dtype == self.tdtype and img.shape[1:] == (IMG, IMG) and img.is_contiguous()
        B = img.shape[0]
        s = self._stream()
        a = torch.empty(B, 128, 128, 64, device=self.device, dtype=self.tdtype)
        if self._dt == _lib.SAD_BF16:
            # one pass: conv1 + batch statistics + sign(gamma)-max-pool, then bn1 + ReLU
            # on the pooled map (conv.hip stem_bf16_kernel<false, true>)
            sz = _lib.SZ()
            _lib.call('sad_stem_train_workspace_size', B, _lib.ctypes.byref(sz))
            ws = self._buf('stem', sz.value)
            st = torch.empty(4 * 64, device=self.device, dtype=torch.float32)
            rm, rv = self.running['bn1'] if self.update_running else (None, None)
            with torch.cuda.device(self.device):
                _lib.call('sad_stem_train_run', _lib.ptr(img), B, _lib.ptr(self.packed('conv1', 4)),
                          _lib.ptr(self.params['bn1.weight']), _lib.ptr(self.params['bn1.bias']), BN_EPS, BN_MOMENTUM,
                          _lib.ptr(rm), _lib.ptr(rv), _lib.ptr(st), _lib.ptr(a), _lib.ptr(ws), ws.numel(), s)
            if self.update_running:
                self.nbt['bn1'] += 1
        else:
            raw = torch.empty(B, 256, 256, 64, device=self.device, dtype=self.tdtype)
            wst = self.packed('conv1', 2)
            chunk = max(1, min(B, stem_chunk))
            col = self._buf('stemcol', chunk * 256 * 256 * 64 * self.es)
            with torch.cuda.device(self.device):
                for i in range(0, B, chunk):
                    n = min(chunk, B - i)
                    _lib.call('sad_stem_conv_run', _lib.ptr(img[i:i + n]), n, IMG, IMG, _lib.ptr(wst), _lib.ptr(col),
                              col.numel(), _lib.ptr(raw[i:i + n]), self._dt, s)
            st = self._bn_stats(raw, 'bn1')
            with torch.cuda.device(self.device):
                _lib.call('sad_bn_relu_maxpool_run', _lib.ptr(raw), B, 256, 256, 64, self._dt, _lib.ptr(st),
                          _lib.ptr(a), s)
            del raw
        return a

    def blocks_fwd(self, a: torch.Tensor, blocks, saved: dict, keep_from: int = 4) -> torch.Tensor:
        """The train-mode blocks ``blocks`` (entries of self.blocks) on a; the
        activations of layer >= keep_from go to ``saved``."""
        if self.bottleneck:
            for blk in blocks:
                a = self._bottleneck_fwd(a, blk, saved, keep_from)
        for prefix, cin, cout, stride, has_ds in ([] if self.bottleneck else blocks):
            c1, st1 = self._conv_bn(a, self.packed(f'{prefix}.conv1', 0), cout, 3, stride, 1, f'{prefix}.bn1')
            a1 = self._bn_apply(c1, st1, relu=True)
            c2, st2 = self._conv_bn(a1, self.packed(f'{prefix}.conv2', 0), cout, 3, 1, 1, f'{prefix}.bn2')
            cd = std = None
            if has_ds:
                cd, std = self._conv_bn(a, self.packed(f'{prefix}.downsample.0', 0), cout, 1, stride, 0,
                                        f'{prefix}.downsample.1')
                out = self._bn_apply(c2, st2, res=cd, rst=std, relu=True)
            else:
                out = self._bn_apply(c2, st2, res=a, relu=True)
            if int(prefix[5]) >= keep_from:
                saved[prefix] = dict(x=a, c1=c1, st1=st1, a1=a1, c2=c2, st2=st2, cd=cd, std=std, out=out)
            a = out
        return a

    def pool(self, a: torch.Tensor) -> torch.Tensor:
        """timm global average pool -> [B, num_features] fp32 (quirk C1's features)."""
        B = a.shape[0]
        feats = torch.empty(B, self.num_features, device=self.device, dtype=torch.float32)
        with torch.cuda.device(self.device):
            _lib.call('sad_avgpool_run', _lib.ptr(a), B, a.shape[1] * a.shape[2], self.num_features, self._dt,
                      _lib.ptr(feats), self._stream())
        return feats

    # ---------------------------------------------------------- backward
    def backward(self, dfeat: torch.Tensor | None, saved: dict, layers=(4,),
                 grads3: Dict[str, torch.Tensor] | None = None, dy: torch.Tensor | None = None,
                 want_dx: bool = False):
        """Gradients of the trainable stages from d(loss)/d(features):
        layer4 into ``self.grads`` (overwritten, as after zero_grad), layer3 (if
        3 in layers) into ``grads3`` (overwritten; the caller folds them into the
        accumulating .grad, quirk C4).  ``dy`` instead of ``dfeat``: the gradient
        of the last block's output (the mixed trainer's hand-over); ``want_dx``:
        also return the gradient of the first processed block's input."""
        order = [b for b in reversed(self.blocks) if int(b[0][5]) in layers]
        if self.bottleneck:
            return self._bottleneck_bwd(dfeat, saved, order, grads3, dy, want_dx)
        dy, dpool = (dy, None) if dy is not None else (None, dfeat)
        for bi, (prefix, cin, cout, stride, has_ds) in enumerate(order):
            sv = saved[prefix]
            G = self.grads if prefix.startswith('layer4') else grads3
            Ho = sv['c2'].shape[1]
            dc2, dz2 = self._bn_backward(sv['c2'], sv['st2'], f'{prefix}.bn2', G, dy=dy, dpool=dpool,
                                         pool_hw=Ho * Ho if dpool is not None else 0, y=sv['out'], want_dz=True)
            dcd = None
            if has_ds:
                dcd, _ = self._bn_backward(sv['cd'], sv['std'], f'{prefix}.downsample.1', G, dy=dz2)
                self._wgrad(sv['x'], dcd, f'{prefix}.downsample.0', G, 1, stride, 0)
            self._wgrad(sv['a1'], dc2, f'{prefix}.conv2', G, 3, 1, 1)
            da1 = self._conv(dc2, self.packed(f'{prefix}.conv2', 1), cout, 3, 1, 1)
            dc1, _ = self._bn_backward(sv['c1'], sv['st1'], f'{prefix}.bn1', G, dy=da1, y=sv['a1'])
            self._wgrad(sv['x'], dc1, f'{prefix}.conv1', G, 3, stride, 1)
            if bi + 1 == len(order) and not want_dx:
                break
            if stride == 1:
                dx = self._conv(dc1, self.packed(f'{prefix}.conv1', 1), cin, 3, 1, 1, res=dz2)
            else:
                dx = torch.empty_like(sv['x'])
                self._dgrad_gemm(dc1, f'{prefix}.conv1', sv['x'].shape, 3, stride, 1, dx, False)
                self._dgrad_gemm(dcd, f'{prefix}.downsample.0', sv['x'].shape, 1, stride, 0, dx, True)
            dy, dpool = dx, None
        return dy if want_dx else None

    # ---------------------------------------------------------- Bottleneck
    def _bottleneck_fwd(self, x, blk, saved, keep_from):
        """timm Bottleneck in train mode: 1x1 -> bn1/ReLU -> 3x3/s -> bn2/ReLU ->
        1x1 -> bn3 (+ downsample 1x1/s + BN, or identity) -> ReLU."""
        prefix, cin, cout, stride, has_ds, width = blk
        c1, st1 = self._conv_bn(x, self.packed(f'{prefix}.conv1', 0), width, 1, 1, 0, f'{prefix}.bn1')
        a1 = self._bn_apply(c1, st1, relu=True)
        c2, st2 = self._conv_bn(a1, self.packed(f'{prefix}.conv2', 0), width, 3, stride, 1, f'{prefix}.bn2')
        a2 = self._bn_apply(c2, st2, relu=True)
        c3, st3 = self._conv_bn(a2, self.packed(f'{prefix}.conv3', 0), cout, 1, 1, 0, f'{prefix}.bn3')
        cd = std = None
        if has_ds:
            cd, std = self._conv_bn(x, self.packed(f'{prefix}.downsample.0', 0), cout, 1, stride, 0,
                                    f'{prefix}.downsample.1')
            out = self._bn_apply(c3, st3, res=cd, rst=std, relu=True)
        else:
            out = self._bn_apply(c3, st3, res=x, relu=True)
        if int(prefix[5]) >= keep_from:
            saved[prefix] = dict(x=x, c1=c1, st1=st1, a1=a1, c2=c2, st2=st2, a2=a2, c3=c3, st3=st3, cd=cd, std=std,
                                 out=out)
        return out

    def _bottleneck_bwd(self, dfeat, saved, order, grads3, dy=None, want_dx=False):
        dy, dpool = (dy, None) if dy is not None else (None, dfeat)
        for bi, (prefix, cin, cout, stride, has_ds, width) in enumerate(order):
            sv = saved[prefix]
            G = self.grads if prefix.startswith('layer4') else grads3
            Ho = sv['c3'].shape[1]
            dc3, dz3 = self._bn_backward(sv['c3'], sv['st3'], f'{prefix}.bn3', G, dy=dy, dpool=dpool,
                                         pool_hw=Ho * Ho if dpool is not None else 0, y=sv['out'], want_dz=True)
            dcd = None
            if has_ds:
                dcd, _ = self._bn_backward(sv['cd'], sv['std'], f'{prefix}.downsample.1', G, dy=dz3)
                self._wgrad(sv['x'], dcd, f'{prefix}.downsample.0', G, 1, stride, 0)
            self._wgrad(sv['a2'], dc3, f'{prefix}.conv3', G, 1, 1, 0)
            da2 = self._conv(dc3, self.packed(f'{prefix}.conv3', 1), width, 1, 1, 0)
            dc2, _ = self._bn_backward(sv['c2'], sv['st2'], f'{prefix}.bn2', G, dy=da2, y=sv['a2'])
            self._wgrad(sv['a1'], dc2, f'{prefix}.conv2', G, 3, stride, 1)
            if stride == 1:
                da1 = self._conv(dc2, self.packed(f'{prefix}.conv2', 1), width, 3, 1, 1)
            else:
                da1 = torch.empty_like(sv['a1'])
                self._dgrad_gemm(dc2, f'{prefix}.conv2', sv['a1'].shape, 3, stride, 1, da1, False)
            dc1, _ = self._bn_backward(sv['c1'], sv['st1'], f'{prefix}.bn1', G, dy=da1, y=sv['a1'])
            self._wgrad(sv['x'], dc1, f'{prefix}.conv1', G, 1, 1, 0)
            if bi + 1 == len(order) and not want_dx:
                break
            # dx = conv1's dgrad (1x1, stride 1) + the shortcut's gradient
            if not has_ds:
                dx = self._conv(dc1, self.packed(f'{prefix}.conv1', 1), cin, 1, 1, 0, res=dz3)
            elif stride == 1:
                dx = self._conv(dc1, self.packed(f'{prefix}.conv1', 1), cin, 1, 1, 0)
                self._dgrad_gemm(dcd, f'{prefix}.downsample.0', sv['x'].shape, 1, 1, 0, dx, True)
            else:
                dx = self._conv(dc1, self.packed(f'{prefix}.conv1', 1), cin, 1, 1, 0)
                self._dgrad_gemm(dcd, f'{prefix}.downsample.0', sv['x'].shape, 1, stride, 0, dx, True)
            dy, dpool = dx, None
        return dy if want_dx else None

    # ---------------------------------------------------------- optimizer
    def clip_grad_norm(self, lo: int, hi: int, max_norm: float = MAX_GRAD_NORM) -> torch.Tensor:
        """clip_grad_norm_ over gflat[lo:hi]; returns device [norm, coef]."""
        nc = torch.empty(2, device=self.device, dtype=torch.float32)
        ws = self._buf('clip', 1024 * 8)
        with torch.cuda.device(self.device):
            _lib.call('sad_clip_grad_norm_run', _lib.ptr(self.gflat[lo:hi]), hi - lo, float(max_norm), _lib.ptr(nc),
                      _lib.ptr(ws), ws.numel(), self._stream())
        return nc

    # ---------------------------------------------------------- --head-loss
    def _head_params(self) -> _lib.HeadParams:
        p, (rm3, rv3), (rm7, rv7) = self.params, self.head_running[3], self.head_running[7]
        t = [p[f'head.{i}.{w}'] for i in (2, 3, 6, 7, 10) for w in ('weight', 'bias')] + [rm3, rv3, rm7, rv7]
        return _lib.HeadParams(*[x.data_ptr() for x in t], self.num_features, BN_EPS, BN_MOMENTUM, *HEAD_DROPOUT)

    def head_forward(self, feats: torch.Tensor, train: bool = True, seed: int = 0) -> torch.Tensor:
        """model.head on the pooled features (sad_head_train_forward_run): train
        mode = batch-statistics BN (running stats updated) + dropout masks of
        ``seed``; eval = running stats, no dropout.  -> logits [B, 2] fp32."""
        B = feats.shape[0]
        sz = _lib.SZ()
        _lib.call('sad_head_workspace_size', B, self.num_features, _lib.ctypes.byref(sz))
        ws = self._buf('head', sz.value)
        logits = torch.empty(B, 2, device=self.device, dtype=torch.float32)
        hp = self._head_params()
        with torch.cuda.device(self.device):
            _lib.call('sad_head_train_forward_run', _lib.ctypes.byref(hp), _lib.ptr(feats.contiguous()), B,
                      int(train), seed & (2 ** 64 - 1), _lib.ptr(logits), _lib.ptr(ws), ws.numel(), self._stream())
        if train:
            for i in (3, 7):
                self.head_nbt[i] += 1
        return logits

    def head_backward(self, feats: torch.Tensor, dlogits: torch.Tensor, seed: int = 0) -> torch.Tensor:
        """After head_forward(train=True) with the same feats and seed: the head's
        parameter gradients into gflat (overwritten) and d(loss)/d(feats)."""
        B = feats.shape[0]
        ws = self._ws['head']
        dfeat = torch.empty(B, self.num_features, device=self.device, dtype=torch.float32)
        a, b = self.range_head
        hp = self._head_params()
        with torch.cuda.device(self.device):
            _lib.call('sad_head_train_backward_run', _lib.ctypes.byref(hp), _lib.ptr(feats.contiguous()), B,
                      seed & (2 ** 64 - 1), _lib.ptr(dlogits.contiguous()), _lib.ptr(dfeat),
                      _lib.ptr(self.gflat[a:b]), _lib.ptr(ws), ws.numel(), self._stream())
        return dfeat

    def current_head_sd(self) -> "OrderedDict[str, torch.Tensor]":
        """model.head's state dict: the trained values under --head-loss, else
        the untouched initial head (quirk C1)."""
        if not self.head_loss:
            return OrderedDict((k, v.clone()) for k, v in self.head_sd.items())
        sd = OrderedDict()
        for k in head_keys():
            i, what = int(k.split('.')[0]), k.split('.', 1)[1]
            if what in ('weight', 'bias'):
                sd[k] = self.params[f'head.{k}'].detach().cpu().clone()
            elif what == 'running_mean':
                sd[k] = self.head_running[i][0].cpu().clone()
            elif what == 'running_var':
                sd[k] = self.head_running[i][1].cpu().clone()
            else:
                sd[k] = torch.tensor(self.head_nbt[i], dtype=torch.long)
        return sd

    # ---------------------------------------------------------- eval / export
    def base_state_dict(self) -> "OrderedDict[str, torch.Tensor]":
        """timm-keyed backbone state dict (CPU), parameters + BN buffers."""
        sd = OrderedDict()
        for key, shape, kind in arch_param_shapes(self.model_name):
            if kind == 'conv':
                sd[f'{key}.weight'] = self.params[f'{key}.weight'].detach().cpu().clone()
            else:
                sd[f'{key}.weight'] = self.params[f'{key}.weight'].detach().cpu().clone()
                sd[f'{key}.bias'] = self.params[f'{key}.bias'].detach().cpu().clone()
                rm, rv = self.running[key]
                sd[f'{key}.running_mean'] = rm.cpu().clone()
                sd[f'{key}.running_var'] = rv.cpu().clone()
                sd[f'{key}.num_batches_tracked'] = torch.tensor(self.nbt[key], dtype=torch.long)
        return sd

    def state_dict(self) -> "OrderedDict[str, torch.Tensor]":
        """``get_model(model).state_dict()`` of the reference trainer: timm keys,
        then ``head.*`` (submodel_trainer.py:706)."""
        sd = self.base_state_dict()
        for k, v in self.current_head_sd().items():
            sd[f'head.{k}'] = v
        return sd

    def eval_backbone(self, micro_batch: int = 64):
        """``model.eval()`` forward: the inference plan (BN folded with the
        current running statistics)."""
        if self.model_name == 'resnet18':
            return Backbone(self.base_state_dict(), self.device, self.dtype, micro_batch)
        return ResNetBackbone(self.base_state_dict(), self.model_name, self.device, self.dtype, micro_batch)


class MixedNet(TrainNet):
    """``--precision mixed``: the frozen prefix (stem, layers 1-3) in fp32 and the
    trained layer4 in bf16, forward and backward.

    The bf16 trainer's layer4 gradients track fp32 autograd only to cosine
    0.93 / 0.70 / 0.62 on resnet50: that is the bf16 rounding of
    layers 1-3's FORWARD activations (CPU emulation, tools/bf16_grad_emulation.py:
    rounding only layer4's forward and backward gives 0.997 / 0.989 / 0.988).
    This net is a bf16 TrainNet (layer4, the packed layer4 weights AdamW
    re-packs, the pool) plus an fp32 TrainNet ``pre`` for the prefix that
    shares every parameter, gradient, running-statistics and counter object;
    the activation crosses with one sad_cast_run each way (layer3's gradient
    comes back through it when layer3 is unfrozen, quirk C4).  The prefix's
    weights never change (layer3 is never stepped), so its fp32 packed copies
    stay valid.  Evaluation runs the split-bf16 inference plan (|dlogit| <= 1e-3)."""

    def __init__(self, base_sd, head_sd, device='cuda', model_name: str = 'resnet18', head_loss: bool = False):
        super().__init__(base_sd, head_sd, device, 'bf16', model_name, head_loss)
        pre = TrainNet.__new__(TrainNet)
        pre.__dict__.update(self.__dict__)
        pre.dtype, pre._dt, pre.tdtype, pre.es = 'fp32', _lib.SAD_F32, torch.float32, 4
        pre._packed, pre._ws = {}, {}
        self.pre = pre
        self.dtype = 'mixed'

    def invalidate_packed(self):
        # both caches: the bf16 layer4 packs and the fp32 prefix packs of ``pre``
        super().invalidate_packed()
        self.pre._packed.clear()

    def _l4(self, blk) -> bool:
        return blk[0].startswith('layer4')

    def _cast(self, x: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
        out = torch.empty(x.shape, device=self.device, dtype=dtype)
        code = {torch.float32: _lib.SAD_F32, torch.bfloat16: _lib.SAD_BF16}
        with torch.cuda.device(self.device):
            _lib.call('sad_cast_run', _lib.ptr(x), code[x.dtype], _lib.ptr(out), code[dtype], x.numel(),
                      self._stream())
        return out

    def forward_train(self, img: torch.Tensor, keep_from: int = 4, stem_chunk: int = 16):
        """img [B, 512, 512] fp32 -> (pooled features fp32, saved activations)."""
        saved = {}
        a = self.pre.stem_fwd(img, stem_chunk)
        a = self.pre.blocks_fwd(a, [b for b in self.blocks if not self._l4(b)], saved, keep_from)
        a = self.blocks_fwd(self._cast(a, torch.bfloat16), [b for b in self.blocks if self._l4(b)], saved, keep_from)
        return self.pool(a), saved

    def backward(self, dfeat, saved, layers=(4,), grads3=None, dy=None, want_dx=False):
        if 3 not in layers:
            return TrainNet.backward(self, dfeat, saved, (4,), grads3)
        dx = TrainNet.backward(self, dfeat, saved, (4,), grads3, want_dx=True)
        return self.pre.backward(None, saved, (3,), grads3, dy=self._cast(dx, torch.float32))

    def eval_backbone(self, micro_batch: int = 64):
        if self.model_name == 'resnet18':
            return Backbone(self.base_state_dict(), self.device, 'bf16x3', micro_batch)
        return ResNetBackbone(self.base_state_dict(), self.model_name, self.device, 'bf16x3', micro_batch)


def ce_loss(feats: torch.Tensor, targets: torch.Tensor, scale: float = 0.0, want_grad: bool = False,
            want_pred: bool = False):
    """(dlogits or None, device [loss_sum, n_correct][, argmax int32 [B]]) of
    CrossEntropyLoss on ``feats`` [B, C] with int64 ``targets`` [B]."""
    B, C = feats.shape
    out = torch.empty(2, device=feats.device, dtype=torch.float32)
    d = torch.empty_like(feats)
    pred = torch.empty(B, device=feats.device, dtype=torch.int32) if want_pred else None
    t = targets.to(feats.device, torch.int64).contiguous()
    with torch.cuda.device(feats.device):
        _lib.call('sad_ce_loss_run', _lib.ptr(feats), _lib.ptr(t), B, C, float(scale), _lib.ptr(d), _lib.ptr(out),
                  _lib.ptr(pred), _lib.stream_handle(feats.device))
    if want_pred:
        return (d if want_grad else None), out, pred
    return (d if want_grad else None), out


class Trainer:
    """One trainer replica: TrainNet + AdamW/clip state + the C4 layer3 gradient
    accumulator, with an optional process group (DDP over RCCL)."""

    def __init__(self, base_sd, head_sd, device='cuda', dtype: str = 'bf16', lr: float = 1e-3, group=None,
                 world: int = 1, model_name: str = 'resnet18', head_loss: bool = False, seed: int = 42):
        """head_loss: CrossEntropy on model.head's two logits (train-mode head,
        trained with layer4) instead of the reference's pooled features (quirk
        C1, the default)."""
        self.net = (MixedNet(base_sd, head_sd, device, model_name, head_loss) if dtype == 'mixed'
                    else TrainNet(base_sd, head_sd, device, dtype, model_name, head_loss))
        self.head_loss = head_loss
        rank = 0
        if world > 1:
            import torch.distributed as dist
            rank = dist.get_rank(group)
        # dropout masks: one stream of counter-hash draws per (seed, rank); step k uses seed_base + k
        self._seed_base = ((seed & 0xFFFFFFFF) << 24) ^ (rank << 56)
        self.device = self.net.device
        self.group, self.world = group, world
        a4, b4 = self.net.range4
        self.m = torch.zeros(b4 - a4, device=self.device, dtype=torch.float32)
        self.v = torch.zeros_like(self.m)
        self.step_count = 0
        self.lr = lr
        self.layer3_unfrozen = False
        self.grads3 = None
        self._g3flat = None
        # torch.optim.AdamW over the same parameter list as the reference
        # (filter(requires_grad): layer4 then head, submodel_trainer.py:648-652) -- used
        # only for state_dict()/load_state_dict() and ReduceLROnPlateau; its step()
        # is never called (sad_adamw_run is the step).
        l4 = [n for n in self.net.names if n.startswith('layer4.')]
        self.l4_names = l4
        # the optimizer's parameters in order: layer4, then the head (stepped only with head_loss)
        self.opt_names = l4 + ([n for n in self.net.names if n.startswith('head.')] if head_loss else [])
        self._head_params = [torch.nn.Parameter(self.net.head_sd[k].clone().float())
                             for k in head_keys() if not k.endswith(('running_mean', 'running_var',
                                                                     'num_batches_tracked'))]
        self._l4_params = [torch.nn.Parameter(self.net.params[n].detach().cpu().clone()) for n in l4]
        self.optimizer = torch.optim.AdamW(self._l4_params + self._head_params, lr=lr, weight_decay=WEIGHT_DECAY)

    # reference: for p in layer3.parameters(): p.requires_grad = True  (:687-691)
    def unfreeze_layer3(self):
        if self.layer3_unfrozen:
            return
        self.layer3_unfrozen = True
        a3, b3 = self.net.range3
        self.net.gflat[a3:b3].zero_()
        self._g3flat = torch.empty(b3 - a3, device=self.device, dtype=torch.float32)
        self.grads3 = OrderedDict()
        for n in self.net.names:
            if n.startswith('layer3.'):
                lo, hi = self.net.offsets[n]
                self.grads3[n] = self._g3flat[lo - a3:hi - a3].view(self.net.params[n].shape)

    @property
    def current_lr(self) -> float:
        return float(self.optimizer.param_groups[-1]['lr'])

    def train_step(self, img: torch.Tensor, targets: torch.Tensor, global_batch: int | None = None):
        """One iteration of submodel_trainer.train()'s batch loop (:253-293).
        ``global_batch`` = rows over all ranks (summed with an all-reduce if
        None).  Returns (mean loss over the global batch, correct count, global
        rows, stepped?)."""
        net = self.net
        if global_batch is None:
            global_batch = img.shape[0]
            if self.world > 1:
                import torch.distributed as dist
                t = torch.tensor([global_batch], device=self.device, dtype=torch.int64)
                dist.all_reduce(t, group=self.group)
                global_batch = int(t.item())
        layers = (3, 4) if self.layer3_unfrozen else (4,)
        feats, saved = net.forward_train(img, keep_from=min(layers))
        if self.head_loss:
            seed = self._seed_base + self.step_count + 1
            logits = net.head_forward(feats, True, seed)
            dlogits, lc = ce_loss(logits, targets, 1.0 / global_batch, want_grad=True)
            dfeat = net.head_backward(feats, dlogits, seed)
        else:
            dfeat, lc = ce_loss(feats, targets, 1.0 / global_batch, want_grad=True)
        if self.world > 1:
            import torch.distributed as dist
            dist.all_reduce(lc, group=self.group)
        # The backward and the gradient all-reduce are queued BEFORE the host
        # reads the loss, so the device never idles on that sync; a NaN/Inf loss
        # (:266-271) then discards them (layer4 grads are overwritten by the next
        # backward, the layer3 step gradient is simply not folded in).
        net.backward(dfeat, saved, layers, self.grads3)
        a4, b4 = net.range4
        if self.world > 1:
            import torch.distributed as dist
            dist.all_reduce(net.gflat[a4:b4], group=self.group)
            if self.layer3_unfrozen:
                dist.all_reduce(self._g3flat, group=self.group)
        loss_sum, correct = lc.tolist()
        loss = loss_sum / global_batch
        if not math.isfinite(loss):  # skip the step
            return loss, 0, 0, False
        lo = a4
        if self.layer3_unfrozen:
            a3, b3 = net.range3
            with torch.cuda.device(self.device):
                _lib.call('sad_axpy_run', _lib.ptr(net.gflat[a3:b3]), _lib.ptr(self._g3flat), b3 - a3, 1.0,
                          _lib.stream_handle(self.device))
            lo = a3
        self.last_norm = net.clip_grad_norm(lo, b4)
        self.step_count += 1
        lr = self.current_lr
        # AdamW, writing the updated layer4 conv weights straight into their cached
        # pack-mode 0 / 1 copies; other cached layouts of layer4 are dropped
        segs = net.pack_segments('layer4.', a4)
        arr = (_lib.PackSeg * max(1, len(segs)))(*segs)
        with torch.cuda.device(self.device):
            _lib.call('sad_adamw_pack_run', _lib.ptr(net.pflat[a4:b4]), _lib.ptr(net.gflat[a4:b4]), _lib.ptr(self.m),
                      _lib.ptr(self.v), b4 - a4, lr, ADAM_BETAS[0], ADAM_BETAS[1], ADAM_EPS, WEIGHT_DECAY,
                      self.step_count, arr, len(segs), net._dt, _lib.stream_handle(self.device))
        net.invalidate('layer4.', keep_modes=(0, 1))
        return loss, int(correct), int(global_batch), True

    # ------------------------------------------------------------ checkpoints
    def optimizer_state_dict(self) -> dict:
        a4, _ = self.net.range4
        st = {}
        if self.step_count:
            for i, n in enumerate(self.opt_names):
                lo, hi = self.net.offsets[n]
                shp = self.net.params[n].shape
                st[i] = {'step': torch.tensor(float(self.step_count)),
                         'exp_avg': self.m[lo - a4:hi - a4].view(shp).cpu().clone(),
                         'exp_avg_sq': self.v[lo - a4:hi - a4].view(shp).cpu().clone()}
        sd = self.optimizer.state_dict()
        sd['state'] = st
        return sd

    def load_optimizer_state_dict(self, sd: dict):
        self.optimizer.load_state_dict(sd)
        a4, _ = self.net.range4
        steps = []
        for i, n in enumerate(self.opt_names):
            s = sd['state'].get(i)
            if not s:
                continue
            lo, hi = self.net.offsets[n]
            self.m[lo - a4:hi - a4].copy_(torch.as_tensor(s['exp_avg']).reshape(-1))
            self.v[lo - a4:hi - a4].copy_(torch.as_tensor(s['exp_avg_sq']).reshape(-1))
            steps.append(int(float(torch.as_tensor(s['step']).item())))
        self.step_count = max(steps) if steps else 0
        self.optimizer.state.clear()

    def load_state_dict(self, sd: dict):
        """``get_model(model).load_state_dict(state_dict)`` (strict) of a trainer checkpoint."""
        net = self.net
        for n in net.names:
            net.params[n].copy_(torch.as_tensor(sd[n], dtype=torch.float32))
        for k in net.bn_keys:
            net.running[k][0].copy_(torch.as_tensor(sd[f'{k}.running_mean']))
            net.running[k][1].copy_(torch.as_tensor(sd[f'{k}.running_var']))
            net.nbt[k] = int(torch.as_tensor(sd[f'{k}.num_batches_tracked']).item())
        for k in head_keys():
            net.head_sd[k] = torch.as_tensor(sd[f'head.{k}']).clone()
        if net.head_loss:
            for i in (3, 7):
                net.head_running[i][0].copy_(torch.as_tensor(sd[f'head.{i}.running_mean']))
                net.head_running[i][1].copy_(torch.as_tensor(sd[f'head.{i}.running_var']))
                net.head_nbt[i] = int(torch.as_tensor(sd[f'head.{i}.num_batches_tracked']).item())
        net.invalidate_packed()
