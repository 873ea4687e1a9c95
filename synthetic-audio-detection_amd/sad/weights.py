"""Deterministic random-init merged checkpoints (no network => no ImageNet weights).

``merged_state_dict(seed, n_heads, distinct_backbones)`` returns a state dict in
the reference's merged-checkpoint layout (``model_merger.py:154-159``;
SURVEY.md Appendix B): ``sub_models.<i>.base.<timm key>`` and
``sub_models.<i>.head.<idx>.<param>``.

Values come from a counter-based hash (sad.synth.mix64) turned into
Irwin-Hall(4) normals with exact float64 arithmetic, so they regenerate
bit-identically on any host.  BatchNorm running statistics default to (0, 1);
tests and the bench overlay calibrated statistics (tests/golden/bn_stats_*.npz)
so that activations stay O(1) through the 20 conv layers.
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import torch

from .synth import GOLD, GOLD2, mix64

BLOCK_CHANNELS = (64, 128, 256, 512)

# timm ResNet variants the reference can name (`--model-name`, submodel_trainer.py:51;
# backbone_name, inference_runner.py:77): block type and blocks per stage.
ARCHS = {
    'resnet18': ('basic', (2, 2, 2, 2)),
    'resnet34': ('basic', (3, 4, 6, 3)),
    'resnet50': ('bottleneck', (3, 4, 6, 3)),
    'resnet101': ('bottleneck', (3, 4, 23, 3)),
    'resnet152': ('bottleneck', (3, 8, 36, 3)),
}


def arch_spec(model_name: str):
    """(block, layers, num_features) of a supported timm ResNet name."""
    if model_name not in ARCHS:
        raise ValueError(f'unsupported backbone {model_name!r} (supported: {", ".join(ARCHS)})')
    block, layers = ARCHS[model_name]
    return block, layers, 512 * (4 if block == 'bottleneck' else 1)


def arch_of_state(base_sd) -> str:
    """The ARCHS name whose timm key set a backbone state dict has (ValueError if none)."""
    keys = {k.rsplit('.', 1)[0] for k in base_sd}
    block = 'bottleneck' if 'layer1.0.conv3' in keys else 'basic'
    layers = tuple(len({k.split('.')[1] for k in keys if k.startswith(f'layer{i}.')}) for i in range(1, 5))
    for name, spec in ARCHS.items():
        if spec == (block, layers):
            return name
    raise ValueError(f'backbone state dict matches no supported ResNet ({block}, {layers})')


def _normals(seed: int, tag: int, n: int) -> np.ndarray:
    key = mix64((mix64(seed & 0xFFFFFFFFFFFFFFFF) + tag * GOLD) & 0xFFFFFFFFFFFFFFFF)
    j = np.arange(n, dtype=np.uint64)
    r = mix64(np.uint64(key) + (j + np.uint64(1)) * np.uint64(GOLD2))
    s = np.zeros(n, dtype=np.int64)
    for sh in (0, 16, 32, 48):
        s += ((r >> np.uint64(sh)) & np.uint64(0xFFFF)).astype(np.int64)
    return (s - 131070).astype(np.float64) / 37837.23


def backbone_param_shapes(layers=(2, 2, 2, 2), block: str = 'basic'):
    """Ordered (timm key, shape, kind) for a BasicBlock or Bottleneck ResNet;
    kind in {conv, bn}.  Mirrors timm's state-dict order (Bottleneck: width =
    planes, expansion 4, stride on conv2)."""
    out = [('conv1', (64, 3, 7, 7), 'conv'), ('bn1', (64,), 'bn')]
    inplanes = 64
    exp = 4 if block == 'bottleneck' else 1
    for li, (planes, n) in enumerate(zip(BLOCK_CHANNELS, layers)):
        for b in range(n):
            s = (1 if li == 0 else 2) if b == 0 else 1
            p = f'layer{li + 1}.{b}'
            if block == 'bottleneck':
                convs = [(planes, inplanes, 1), (planes, planes, 3), (planes * exp, planes, 1)]
            else:
                convs = [(planes, inplanes, 3), (planes, planes, 3)]
            for j, (co, ci, k) in enumerate(convs):
                out.append((f'{p}.conv{j + 1}', (co, ci, k, k), 'conv'))
                out.append((f'{p}.bn{j + 1}', (co,), 'bn'))
            if b == 0 and (s != 1 or inplanes != planes * exp):
                out.append((f'{p}.downsample.0', (planes * exp, inplanes, 1, 1), 'conv'))
                out.append((f'{p}.downsample.1', (planes * exp,), 'bn'))
            inplanes = planes * exp
    return out


def arch_param_shapes(model_name: str = 'resnet18'):
    block, layers, _ = arch_spec(model_name)
    return backbone_param_shapes(layers, block)


HEAD_LAYOUT = [(2, 'linear', (512, 512)), (3, 'bn', (512,)), (6, 'linear', (256, 512)),
               (7, 'bn', (256,)), (10, 'linear', (2, 256))]


def head_layout(num_features: int = 512):
    """HEAD_LAYOUT with the first Linear's input width = the backbone's num_features."""
    return [(2, 'linear', (512, num_features))] + HEAD_LAYOUT[1:]


def _bn(seed, tag, c, prefix, sd):
    sd[f'{prefix}.weight'] = torch.from_numpy((1.0 + 0.1 * _normals(seed, tag, c)).astype(np.float32))
    sd[f'{prefix}.bias'] = torch.from_numpy((0.1 * _normals(seed, tag + 1, c)).astype(np.float32))
    sd[f'{prefix}.running_mean'] = torch.zeros(c)
    sd[f'{prefix}.running_var'] = torch.ones(c)
    sd[f'{prefix}.num_batches_tracked'] = torch.tensor(0, dtype=torch.long)


def backbone_state_dict(seed: int, model_name: str = 'resnet18') -> "OrderedDict[str, torch.Tensor]":
    sd = OrderedDict()
    for t, (key, shape, kind) in enumerate(arch_param_shapes(model_name)):
        tag = 1000 + 4 * t
        if kind == 'conv':
            fan_out = shape[0] * shape[2] * shape[3]
            std = (2.0 / fan_out) ** 0.5
            w = (_normals(seed, tag, int(np.prod(shape))) * std).astype(np.float32).reshape(shape)
            sd[f'{key}.weight'] = torch.from_numpy(w)
        else:
            _bn(seed, tag, shape[0], key, sd)
    return sd


def head_state_dict(seed: int, num_features: int = 512) -> "OrderedDict[str, torch.Tensor]":
    sd = OrderedDict()
    for t, (idx, kind, shape) in enumerate(head_layout(num_features)):
        tag = 9000 + 4 * t
        if kind == 'linear':
            fan_in = shape[1]
            w = (_normals(seed, tag, shape[0] * shape[1]) / np.sqrt(fan_in)).astype(np.float32)
            sd[f'{idx}.weight'] = torch.from_numpy(w.reshape(shape))
            sd[f'{idx}.bias'] = torch.from_numpy((0.05 * _normals(seed, tag + 1, shape[0])).astype(np.float32))
        else:
            _bn(seed, tag, shape[0], str(idx), sd)
    return sd


def empty_state_dicts(model_name: str = 'resnet18'):
    """(backbone, head) state dicts with the right keys/shapes and placeholder
    values (zeros; BN var = 1) -- the cheap skeleton a checkpoint is loaded into."""
    nf = arch_spec(model_name)[2]
    bb = OrderedDict()
    for key, shape, kind in arch_param_shapes(model_name):
        if kind == 'conv':
            bb[f'{key}.weight'] = torch.zeros(shape)
        else:
            c = shape[0]
            bb[f'{key}.weight'], bb[f'{key}.bias'] = torch.ones(c), torch.zeros(c)
            bb[f'{key}.running_mean'], bb[f'{key}.running_var'] = torch.zeros(c), torch.ones(c)
            bb[f'{key}.num_batches_tracked'] = torch.tensor(0, dtype=torch.long)
    hd = OrderedDict()
    for idx, kind, shape in head_layout(nf):
        if kind == 'linear':
            hd[f'{idx}.weight'], hd[f'{idx}.bias'] = torch.zeros(shape), torch.zeros(shape[0])
        else:
            c = shape[0]
            hd[f'{idx}.weight'], hd[f'{idx}.bias'] = torch.ones(c), torch.zeros(c)
            hd[f'{idx}.running_mean'], hd[f'{idx}.running_var'] = torch.zeros(c), torch.ones(c)
            hd[f'{idx}.num_batches_tracked'] = torch.tensor(0, dtype=torch.long)
    return bb, hd


def merged_state_dict(seed: int = 0, n_heads: int = 6, distinct_backbones: bool = False,
                      bn_stats: dict | None = None, model_name: str = 'resnet18') -> "OrderedDict[str, torch.Tensor]":
    """Merged checkpoint state dict.  Sub-model i uses backbone seed
    ``seed + (i if distinct_backbones else 0)`` (shared backbone = the reference's
    quirk C2 situation) and head seed ``seed * 1000 + i + 1``.  ``bn_stats`` maps
    full keys (``sub_models.i....running_mean``) to arrays overriding defaults."""
    sd = OrderedDict()
    cache = {}
    for i in range(n_heads):
        bseed = seed + (i if distinct_backbones else 0)
        if bseed not in cache:
            cache[bseed] = backbone_state_dict(bseed, model_name)
        bb = cache[bseed]
        for k, v in bb.items():
            sd[f'sub_models.{i}.base.{k}'] = v.clone()
        hd = head_state_dict(seed * 1000 + i + 1, arch_spec(model_name)[2])
        for k, v in hd.items():
            sd[f'sub_models.{i}.head.{k}'] = v.clone()
    if bn_stats:
        for k, v in bn_stats.items():
            if k in sd:
                sd[k] = torch.as_tensor(np.asarray(v), dtype=sd[k].dtype).reshape(sd[k].shape)
    return sd


def load_bn_stats(path) -> dict:
    z = np.load(path, allow_pickle=False)
    return {k: z[k] for k in z.files}
