"""Device engine: front end, backbone(s) and heads as libsad plans.

This is the MI355X replacement of the reference's device work:
  * ``FrontEnd``  -- torchaudio MelSpectrogram/AmplitudeToDB + standardise
    (inference_runner.py:157-171; trainer norm=None variant
    submodel_trainer.py:97-105,191-199)
  * ``Backbone``  -- timm resnet18 forward_features + AdaptiveAvgPool2d
    (inference_runner.py:35,37,49-51), with Resize((512,512)) + repeat(3)
    (:172-174) fused into the stem
  * ``ResNetBackbone`` -- the deeper timm names (resnet34/50/101/152,
    SURVEY.md 8(f) row 4) on the same kernels (libsad sad_resnet_*)
  * ``Heads``     -- BinaryClassifier.head x N + ModularMultiHeadClassifier
    merge (inference_runner.py:36-48,62-73)
  * ``Engine``    -- a merged checkpoint's state dict -> the three above.
    Sub-models whose ``base.*`` tensors are identical (the reference's quirk
    C2 makes that the normal case) share ONE backbone run.

Every call is asynchronous on torch's current stream of the engine's device.
"""
from __future__ import annotations

import hashlib
from typing import Dict, List, Sequence

import numpy as np
import torch

from . import _lib
from .weights import arch_of_state, arch_param_shapes, arch_spec, backbone_param_shapes

MAP_H, MAP_W = 128, 251
N_SAMPLES = 128000
HEAD_KEYS = ['2.weight', '2.bias', '3.weight', '3.bias', '3.running_mean', '3.running_var',
             '6.weight', '6.bias', '7.weight', '7.bias', '7.running_mean', '7.running_var',
             '10.weight', '10.bias']


def _dev(device) -> torch.device:
    d = torch.device(device)
    if d.type != 'cuda':
        raise RuntimeError(f'libsad runs on MI355X devices only (got {d}); there is no CPU path')
    return torch.device('cuda', d.index if d.index is not None else torch.cuda.current_device())


def _np32(t) -> np.ndarray:
    return np.ascontiguousarray(torch.as_tensor(t).detach().to('cpu', torch.float32).numpy())


def _checked(sd: Dict[str, torch.Tensor], key: str, shape) -> np.ndarray:
    """sd[key] as contiguous fp32, after checking its shape: the C plan builders
    read raw host pointers with the layout's sizes, so a wrong width (e.g. a
    wide_resnet state dict) must fail here, not overrun host memory there."""
    if key not in sd:
        raise KeyError(f'missing tensor {key!r}')
    a = _np32(sd[key])
    if tuple(a.shape) != tuple(shape):
        raise ValueError(f'tensor {key!r} has shape {tuple(a.shape)}, expected {tuple(shape)}')
    return a


def _backbone_arrays(base_sd, shapes) -> list:
    arrays = []
    for key, shape, kind in shapes:
        if kind == 'conv':
            arrays.append(_checked(base_sd, f'{key}.weight', shape))
        else:
            for s in ('weight', 'bias', 'running_mean', 'running_var'):
                arrays.append(_checked(base_sd, f'{key}.{s}', shape))
    return arrays


def _head_arrays(sd, num_features: int) -> list:
    from .weights import head_layout
    shapes = {}
    for idx, kind, shape in head_layout(num_features):
        if kind == 'linear':
            shapes[f'{idx}.weight'], shapes[f'{idx}.bias'] = shape, shape[:1]
        else:
            for s in ('weight', 'bias', 'running_mean', 'running_var'):
                shapes[f'{idx}.{s}'] = shape
    return [_checked(sd, k, shapes[k]) for k in HEAD_KEYS]


class FrontEnd:
    def __init__(self, device='cuda', norm: str | None = 'slaney', n_samples: int = N_SAMPLES,
                 sample_rate: int = 32000, n_fft: int = 2048, hop: int = 512, n_mels: int = 128,
                 f_min: float = 20.0, f_max: float = 12000.0, top_db: float | None = 80.0):
        self.device = _dev(device)
        cfg = _lib.FrontendCfg(sample_rate, n_fft, hop, n_mels, f_min, f_max, 1 if norm == 'slaney' else 0,
                               -1.0 if top_db is None else float(top_db), n_samples)
        self._plan = _lib.P()
        # torchaudio's own fp32 filterbank (sad.audio.melscale_fbanks), not the
        # library's float64 rounding of the same triangles
        from .audio import melscale_fbanks
        fb = melscale_fbanks(n_fft // 2 + 1, float(f_min), float(f_max), n_mels, sample_rate,
                             norm == 'slaney').contiguous()
        # the plan reads a host fp32 [n_freqs, n_mels] array through this pointer
        assert fb.dtype == torch.float32 and fb.device.type == 'cpu' and fb.is_contiguous()
        with torch.cuda.device(self.device):
            _lib.call('sad_frontend_plan_create_fb', _lib.ctypes.byref(cfg), fb.data_ptr(),
                      _lib.ctypes.byref(self._plan))
        nf = _lib.I32()
        _lib.call('sad_frontend_frames', self._plan, _lib.ctypes.byref(nf))
        self.n_frames, self.n_mels, self.n_samples = nf.value, n_mels, n_samples

    def __call__(self, pcm: torch.Tensor, want_db: bool = False, out: torch.Tensor | None = None):
        """pcm [n, >=n_samples] int16 (or fp32 waveform in [-1,1)) on device ->
        map [n, n_mels, frames] fp32 (and the clamped dB map if want_db)."""
        assert pcm.dtype in (torch.int16, torch.float32) and pcm.device == self.device and pcm.dim() == 2
        assert pcm.stride(1) == 1 and pcm.shape[1] >= self.n_samples
        n = pcm.shape[0]
        if out is None:
            out = torch.empty(n, self.n_mels, self.n_frames, device=self.device, dtype=torch.float32)
        db = torch.empty_like(out) if want_db else None
        fn = 'sad_frontend_run' if pcm.dtype == torch.int16 else 'sad_frontend_run_f32'
        with torch.cuda.device(self.device):
            _lib.call(fn, self._plan, _lib.ptr(pcm), n, pcm.stride(0), _lib.ptr(db), _lib.ptr(out),
                      _lib.stream_handle(self.device))
        return (out, db) if want_db else out

    def windows(self, wf: torch.Tensor, offsets: torch.Tensor, want_db: bool = False,
                out: torch.Tensor | None = None):
        """Windows of one long fp32 waveform wf [T] on the device, segment i at
        sample offsets[i] (int64 device tensor), read in place
        (sad_frontend_run_windows) -> map [n, n_mels, frames]."""
        assert wf.dtype == torch.float32 and wf.dim() == 1 and wf.is_contiguous() and wf.device == self.device
        assert offsets.dtype == torch.int64 and offsets.dim() == 1 and offsets.is_contiguous()
        assert offsets.device == self.device and wf.shape[0] >= self.n_samples
        n = offsets.shape[0]
        if out is None:
            out = torch.empty(n, self.n_mels, self.n_frames, device=self.device, dtype=torch.float32)
        db = torch.empty_like(out) if want_db else None
        with torch.cuda.device(self.device):
            _lib.call('sad_frontend_run_windows', self._plan, _lib.ptr(wf), wf.shape[0], _lib.ptr(offsets), n,
                      _lib.ptr(db), _lib.ptr(out), _lib.stream_handle(self.device))
        return (out, db) if want_db else out

    def __del__(self):
        try:
            if getattr(self, '_plan', None):
                _lib.load().sad_frontend_plan_destroy(self._plan)
        except Exception:
            pass


def _dtype_code(dtype: str) -> int:
    if dtype not in _lib.DTYPES:
        raise ValueError(f'dtype must be one of {sorted(_lib.DTYPES)} (got {dtype!r})')
    return _lib.DTYPES[dtype]


def to_split(x: torch.Tensor) -> torch.Tensor:
    """fp32 [..., C] -> the split-bf16 layout [..., 2C] bf16 of dtype 'bf16x3':
    per group of 32 channels [hi(32) | lo(32)], hi = bf16(x), lo = bf16(x - hi)."""
    C = x.shape[-1]
    assert C % 32 == 0
    hi = x.to(torch.bfloat16)
    lo = (x - hi.float()).to(torch.bfloat16)
    g = torch.stack([hi.reshape(*x.shape[:-1], C // 32, 32), lo.reshape(*x.shape[:-1], C // 32, 32)], dim=-2)
    return g.reshape(*x.shape[:-1], 2 * C).contiguous()


def from_split(t: torch.Tensor) -> torch.Tensor:
    """The split-bf16 layout [..., 2C] bf16 -> fp32 [..., C] (hi + lo)."""
    C2 = t.shape[-1]
    g = t.reshape(*t.shape[:-1], C2 // 64, 2, 32).float()
    return (g[..., 0, :] + g[..., 1, :]).reshape(*t.shape[:-1], C2 // 2)


def _act_channels(dtype: str, c: int) -> int:
    return 2 * c if dtype == 'bf16x3' else c


def resize(map_: torch.Tensor, size=(512, 512), dtype: str = 'fp32') -> torch.Tensor:
    """Device bilinear resize (torchvision Resize semantics) of [n, h, w] fp32."""
    n, h, w = map_.shape
    dt = _lib.SAD_BF16 if dtype == 'bf16' else _lib.SAD_F32  # resize output: fp32 or bf16 image
    out = torch.empty(n, size[0], size[1], device=map_.device,
                      dtype=torch.bfloat16 if dt == _lib.SAD_BF16 else torch.float32)
    with torch.cuda.device(map_.device):
        _lib.call('sad_resize_run', _lib.ptr(map_.contiguous()), n, h, w, size[0], size[1], dt, _lib.ptr(out),
                  _lib.stream_handle(map_.device))
    return out


class Backbone:
    """One ResNet-18 backbone; ``base_sd`` uses timm keys (conv1.weight, ...)."""

    def __init__(self, base_sd: Dict[str, torch.Tensor], device='cuda', dtype: str = 'bf16',
                 micro_batch: int = 64):
        self.device = _dev(device)
        self.dtype = dtype
        self._dt = _dtype_code(dtype)
        self.tdtype = torch.float32 if dtype == 'fp32' else torch.bfloat16
        self.micro_batch = micro_batch
        arrays = _backbone_arrays(base_sd, backbone_param_shapes())
        self._plan = _lib.P()
        with torch.cuda.device(self.device):
            # the plan copies (hipMemcpy, synchronous) what it needs; the host arrays die here
            _lib.call('sad_backbone_plan_create', _lib.pointer_array(arrays), len(arrays), self._dt, MAP_H, MAP_W,
                      _lib.ctypes.byref(self._plan))
        self._ws = None

    def workspace(self, mb: int) -> torch.Tensor:
        sz = _lib.SZ()
        _lib.call('sad_backbone_workspace_size', self._plan, mb, _lib.ctypes.byref(sz))
        if self._ws is None or self._ws.numel() < sz.value:
            self._ws = torch.empty(sz.value, dtype=torch.uint8, device=self.device)
        return self._ws

    def __call__(self, maps: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        assert maps.dtype == torch.float32 and maps.shape[1:] == (MAP_H, MAP_W) and maps.is_contiguous()
        B = maps.shape[0]
        feats = out if out is not None else torch.empty(B, 512, device=self.device, dtype=torch.float32)
        mb = max(1, min(self.micro_batch, B))
        ws = self.workspace(mb)
        with torch.cuda.device(self.device):
            _lib.call('sad_backbone_run', self._plan, _lib.ptr(maps), B, mb, _lib.ptr(feats), _lib.ptr(ws),
                      ws.numel(), _lib.stream_handle(self.device))
        return feats

    def forward_images(self, img: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """img [B,512,512] fp32 (one channel of the reference's identical three) -> feats."""
        assert img.dtype == torch.float32 and img.shape[1:] == (512, 512) and img.is_contiguous()
        B = img.shape[0]
        feats = out if out is not None else torch.empty(B, 512, device=self.device, dtype=torch.float32)
        mb = max(1, min(self.micro_batch, B))
        ws = self.workspace(mb)
        with torch.cuda.device(self.device):
            _lib.call('sad_backbone_run_img', self._plan, _lib.ptr(img), B, mb, _lib.ptr(feats), _lib.ptr(ws),
                      ws.numel(), _lib.stream_handle(self.device))
        return feats

    def forward_images3(self, img3: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """img3 [B,3,512,512] fp32 with possibly distinct channels -> feats [B,512]."""
        assert img3.dtype == torch.float32 and img3.shape[1:] == (3, 512, 512) and img3.is_contiguous()
        B = img3.shape[0]
        feats = out if out is not None else torch.empty(B, 512, device=self.device, dtype=torch.float32)
        mb = max(1, min(self.micro_batch, B))
        ws = self.workspace(mb)
        with torch.cuda.device(self.device):
            _lib.call('sad_backbone_run_img3', self._plan, _lib.ptr(img3), B, mb, _lib.ptr(feats), _lib.ptr(ws),
                      ws.numel(), _lib.stream_handle(self.device))
        return feats

    def stem(self, maps: torch.Tensor) -> torch.Tensor:
        """NHWC [B,128,128,64] in the plan dtype (bf16x3: fp32 decoded from the split layout)."""
        B = maps.shape[0]
        out = torch.empty(B, 128, 128, _act_channels(self.dtype, 64), device=self.device, dtype=self.tdtype)
        with torch.cuda.device(self.device):
            _lib.call('sad_backbone_stem_run', self._plan, _lib.ptr(maps.contiguous()), B, _lib.ptr(out),
                      _lib.stream_handle(self.device))
        return from_split(out) if self.dtype == 'bf16x3' else out

    def debug(self, maps: torch.Tensor):
        """(pooled feats [B,512], layer4 map NHWC [B,16,16,512]) for small B."""
        B = maps.shape[0]
        feats = torch.empty(B, 512, device=self.device, dtype=torch.float32)
        l4 = torch.empty(B, 16, 16, _act_channels(self.dtype, 512), device=self.device, dtype=self.tdtype)
        ws = self.workspace(B)
        with torch.cuda.device(self.device):
            _lib.call('sad_backbone_run_debug', self._plan, _lib.ptr(maps.contiguous()), B, _lib.ptr(feats),
                      _lib.ptr(l4), _lib.ptr(ws), ws.numel(), _lib.stream_handle(self.device))
        return feats, (from_split(l4) if self.dtype == 'bf16x3' else l4)

    def __del__(self):
        try:
            if getattr(self, '_plan', None):
                _lib.load().sad_backbone_plan_destroy(self._plan)
        except Exception:
            pass


class ResNetBackbone:
    """A timm resnet34/50/101/152 backbone (``base_sd`` in timm keys) on the
    generic libsad ResNet plan: map -> pooled [B, num_features] fp32."""

    def __init__(self, base_sd: Dict[str, torch.Tensor], model_name: str, device='cuda', dtype: str = 'bf16',
                 micro_batch: int = 64):
        self.device = _dev(device)
        self.dtype = dtype
        self.model_name = model_name
        block, layers, self.num_features = arch_spec(model_name)
        self._dt = _dtype_code(dtype)
        # operands past the kernels' 2 GiB buffer range run as several launches
        # over image ranges (launch_block_conv), so the micro-batch is free
        self.micro_batch = max(1, micro_batch)
        arrays = _backbone_arrays(base_sd, arch_param_shapes(model_name))
        lay = (_lib.I32 * 4)(*layers)
        self._plan = _lib.P()
        with torch.cuda.device(self.device):
            _lib.call('sad_resnet_plan_create', _lib.pointer_array(arrays), len(arrays),
                      1 if block == 'bottleneck' else 0, lay, self._dt, MAP_H, MAP_W, _lib.ctypes.byref(self._plan))
        self._ws = None

    def _run(self, fn: str, x: torch.Tensor, out: torch.Tensor | None) -> torch.Tensor:
        B = x.shape[0]
        feats = out if out is not None else torch.empty(B, self.num_features, device=self.device,
                                                        dtype=torch.float32)
        mb = max(1, min(self.micro_batch, B))
        sz = _lib.SZ()
        _lib.call('sad_resnet_workspace_size', self._plan, mb, _lib.ctypes.byref(sz))
        if self._ws is None or self._ws.numel() < sz.value:
            self._ws = torch.empty(sz.value, dtype=torch.uint8, device=self.device)
        with torch.cuda.device(self.device):
            _lib.call(fn, self._plan, _lib.ptr(x), B, mb, _lib.ptr(feats), _lib.ptr(self._ws),
                      self._ws.numel(), _lib.stream_handle(self.device))
        return feats

    def __call__(self, maps: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        assert maps.dtype == torch.float32 and maps.shape[1:] == (MAP_H, MAP_W) and maps.is_contiguous()
        return self._run('sad_resnet_run', maps, out)

    def forward_images(self, img: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """img [B,512,512] fp32 (one channel of the reference's identical three) -> feats."""
        assert img.dtype == torch.float32 and img.shape[1:] == (512, 512) and img.is_contiguous()
        return self._run('sad_resnet_run_img', img, out)

    def forward_images3(self, img3: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """img3 [B,3,512,512] fp32 with possibly distinct channels -> feats."""
        assert img3.dtype == torch.float32 and img3.shape[1:] == (3, 512, 512) and img3.is_contiguous()
        return self._run('sad_resnet_run_img3', img3, out)

    def __del__(self):
        try:
            if getattr(self, '_plan', None):
                _lib.load().sad_resnet_plan_destroy(self._plan)
        except Exception:
            pass


class Heads:
    """N BinaryClassifier heads (+ merge); ``head_sds[h]`` uses nn.Sequential
    index keys (2.weight, 3.running_mean, ...)."""

    def __init__(self, head_sds: Sequence[Dict[str, torch.Tensor]], feat_index: Sequence[int], n_feat: int,
                 device='cuda', feat_dim: int = 512):
        self.device = _dev(device)
        self.n_heads = len(head_sds)
        arrays = [a for sd in head_sds for a in _head_arrays(sd, feat_dim)]
        fi = (_lib.I32 * self.n_heads)(*feat_index)
        self._plan = _lib.P()
        with torch.cuda.device(self.device):
            _lib.call('sad_heads_plan_create_dim', _lib.pointer_array(arrays), self.n_heads, fi, n_feat,
                      feat_dim, _lib.ctypes.byref(self._plan))
        self.n_feat = n_feat
        self._ws = None

    def __call__(self, feats: Sequence[torch.Tensor], logits: torch.Tensor | None = None,
                 merged: torch.Tensor | None = None):
        B = feats[0].shape[0]
        if logits is None:
            logits = torch.empty(B, self.n_heads, 2, device=self.device, dtype=torch.float32)
        if merged is None:
            merged = torch.empty(B, self.n_heads + 1, device=self.device, dtype=torch.float32)
        sz = _lib.SZ()
        _lib.call('sad_heads_workspace_size', self._plan, B, _lib.ctypes.byref(sz))
        if self._ws is None or self._ws.numel() < sz.value:
            self._ws = torch.empty(sz.value, dtype=torch.uint8, device=self.device)
        fp = (_lib.ctypes.c_void_p * self.n_feat)(*[f.data_ptr() for f in feats])
        with torch.cuda.device(self.device):
            _lib.call('sad_heads_merge_run', self._plan, fp, B, _lib.ptr(logits), _lib.ptr(merged),
                      _lib.ptr(self._ws), self._ws.numel(), _lib.stream_handle(self.device))
        return logits, merged

    def __del__(self):
        try:
            if getattr(self, '_plan', None):
                _lib.load().sad_heads_plan_destroy(self._plan)
        except Exception:
            pass


def _arch(base_sd) -> str:
    """Architecture name of a backbone state dict.  A BasicBlock key set that
    matches no depth is treated as resnet18 so that the missing-key check names
    what is absent; a Bottleneck key set (conv3 keys) that matches no depth
    raises -- read as resnet18 its 1x1 convs would be taken for 3x3."""
    if not base_sd:
        return 'resnet18'
    try:
        return arch_of_state(base_sd)
    except ValueError:
        if any('.conv3.' in k for k in base_sd):
            raise
        return 'resnet18'


def _digest(tensors: List[torch.Tensor]) -> str:
    h = hashlib.sha1()
    for t in tensors:
        h.update(_np32(t).tobytes())
    return h.hexdigest()


def split_merged_state(sd: Dict[str, torch.Tensor]):
    """merged state dict -> (sorted sub-model indices, {i: base_sd}, {i: head_sd}).
    Index parsing follows inference_runner.py:88-98 (sorted ints after
    ``sub_models.``)."""
    idx = set()
    for k in sd.keys():
        parts = k.split('.')
        if len(parts) >= 3 and parts[0] == 'sub_models':
            try:
                idx.add(int(parts[1]))
            except ValueError:
                pass
    idx = sorted(idx)
    bases, heads = {}, {}
    for i in idx:
        pre = f'sub_models.{i}.'
        bases[i] = {k[len(pre) + 5:]: v for k, v in sd.items() if k.startswith(pre + 'base.')}
        heads[i] = {k[len(pre) + 5:]: v for k, v in sd.items() if k.startswith(pre + 'head.')}
    return idx, bases, heads


class Engine:
    """Merged checkpoint -> device pipeline  pcm -> (per-head logits, merged)."""

    def __init__(self, merged_sd: Dict[str, torch.Tensor], device='cuda', dtype: str = 'bf16',
                 micro_batch: int = 64, norm: str | None = 'slaney'):
        self.device = _dev(device)
        self.dtype = dtype
        idx, bases, heads = split_merged_state(merged_sd)
        if not idx:
            raise ValueError('state dict has no sub_models.<i>.* keys')
        self.indices = idx
        digests, self.backbones, feat_index = {}, [], []
        archs = {_arch(bases[i]) for i in idx}
        if len(archs) != 1:
            raise ValueError(f'sub-models mix backbone architectures {sorted(archs)}')
        self.arch = archs.pop()
        for i in idx:
            keys = [k for k, _, kind in arch_param_shapes(self.arch)]
            missing = [k for k in keys if not any(s.startswith(k + '.') for s in bases[i])]
            if missing:
                raise KeyError(f'sub-model {i} lacks backbone tensors {missing[:3]}...')
            d = _digest([bases[i][k] for k in sorted(bases[i]) if not k.endswith('num_batches_tracked')])
            if d not in digests:
                digests[d] = len(self.backbones)
                if self.arch == 'resnet18':  # the tuned ResNet-18 plan
                    self.backbones.append(Backbone(bases[i], self.device, dtype, micro_batch))
                else:
                    self.backbones.append(ResNetBackbone(bases[i], self.arch, self.device, dtype, micro_batch))
            feat_index.append(digests[d])
        self.num_features = arch_spec(self.arch)[2]
        self.heads = Heads([heads[i] for i in idx], feat_index, len(self.backbones), self.device,
                           feat_dim=self.num_features)
        self.frontend = FrontEnd(self.device, norm=norm)
        self.n_heads = len(idx)

    def forward_maps(self, maps: torch.Tensor):
        feats = [bb(maps) for bb in self.backbones]
        return self.heads(feats)

    def forward_pcm(self, pcm: torch.Tensor):
        return self.forward_maps(self.frontend(pcm))


def conv2d(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, stride: int = 1, pad: int = 0,
           res: torch.Tensor | None = None, relu: bool = True, variant: int = 0,
           out: torch.Tensor | None = None) -> torch.Tensor:
    """NHWC conv on the libsad implicit-GEMM kernel.  x [N,H,W,Cin] bf16|fp32,
    w [Cout,k,k,Cin] same dtype, bias [Cout] fp32, res [N,Ho,Wo,Cout] or None."""
    N, H, W, Cin = x.shape
    Cout, k = w.shape[0], w.shape[1]
    Ho, Wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    dt = _lib.SAD_BF16 if x.dtype == torch.bfloat16 else _lib.SAD_F32
    if out is None:
        out = torch.empty(N, Ho, Wo, Cout, device=x.device, dtype=x.dtype)
    with torch.cuda.device(x.device):
        _lib.call('sad_conv2d_run', _lib.ptr(x), N, H, W, Cin, _lib.ptr(w), _lib.ptr(bias), _lib.ptr(res),
                  _lib.ptr(out), Cout, k, stride, pad, int(relu), dt, variant, _lib.stream_handle(x.device))
    return out


def block_conv(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, stride: int = 1, pad: int = 1,
               sc: torch.Tensor | None = None, sc_stride: int = 1, relu: bool = True, variant: int = 0,
               out: torch.Tensor | None = None, res: torch.Tensor | None = None, k: int = 3,
               split: bool = False, four: bool = False) -> torch.Tensor:
    """conv(x) + 1x1 shortcut(sc) [+ res] as ONE launch (libsad block-conv kernels).
    split=True: every tensor in the split-bf16 layout (``to_split``; dtype 'bf16x3');
    four=True (with split): the four-product form of the deep Bottleneck plans.
    x [N,H,W,Cin], sc [N,H1,W1,Cin1] or None, w [Cout, wt_ld] with the k*k*Cin
    conv taps first and the shortcut's Cin1 columns next (extra columns are
    ignored), bias [Cout] fp32, res [N,Ho,Wo,Cout] (epilogue identity shortcut)."""
    N, H, W, Cin = x.shape
    Cout = w.shape[0]
    Cin1 = sc.shape[3] if sc is not None else 0
    Ho, Wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    dt = _lib.SAD_BF16 if x.dtype == torch.bfloat16 else _lib.SAD_F32
    if split:  # x, sc, res, out, w in the split-bf16 layout; channel counts are logical
        dt = _lib.SAD_BF16X3
        Cin, Cin1, wt_ld = Cin // 2, Cin1 // 2, w.stride(0) // 2
    else:
        wt_ld = w.stride(0)
    if out is None:
        out = torch.empty(N, Ho, Wo, _act_channels('bf16x3' if split else 'bf16', Cout), device=x.device,
                          dtype=x.dtype)
    H1, W1 = (sc.shape[1], sc.shape[2]) if sc is not None else (0, 0)
    with torch.cuda.device(x.device):
        _lib.call('sad_block_conv_run', _lib.ptr(x), N, H, W, Cin, _lib.ptr(sc), H1, W1, Cin1, sc_stride,
                  _lib.ptr(w), wt_ld, _lib.ptr(bias), _lib.ptr(res), _lib.ptr(out), Cout, k, stride, pad,
                  int(relu), dt, variant | (_lib.SAD_CONV_FOUR_PRODUCTS if four else 0),
                  _lib.stream_handle(x.device))
    return out
