"""Oracle ResNet-18 backbone + BinaryClassifier head + ensemble merge (fp32, CPU).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

* ``ResNet`` restates ``timm.create_model('resnet18', num_classes=0)`` as called
  at ``inference_runner.py:35`` / ``model_merger.py:24`` /
  ``submodel_trainer.py:606`` (and the deeper names those call sites accept:
  resnet34 BasicBlocks; resnet50/101/152 Bottlenecks, timm's v1.5 layout with
  the stride on the 3x3 conv): BasicBlock ResNet, conv1 7x7/2 + bn1 + act1 +
  maxpool 3x3/2, layer1..4, 1x1/2 conv + BN downsample; ``forward_features``
  returns the layer4 map.  Parameter/buffer names match timm's state-dict keys
   so reference checkpoints load unchanged.
* ``BinaryClassifier`` restates ``inference_runner.py:28-51``
  (== ``model_merger.py:18-40``).
* ``ModularMultiHeadClassifier`` restates ``inference_runner.py:53-73``
  (== ``model_merger.py:61-91``).
"""
from __future__ import annotations

from typing import List

import torch
import torch.nn as nn


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: nn.Module | None = None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.act1 = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=1, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.act2 = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        shortcut = x
        x = self.act1(self.bn1(self.conv1(x)))
        x = self.bn2(self.conv2(x))
        if self.downsample is not None:
            shortcut = self.downsample(shortcut)
        x = x + shortcut
        return self.act2(x)


class Bottleneck(nn.Module):
    """timm Bottleneck (resnet50/101/152): 1x1 -> 3x3/s -> 1x1 (x4), width = planes."""
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: nn.Module | None = None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.act1 = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.act2 = nn.ReLU(inplace=True)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.act3 = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        shortcut = x
        x = self.act1(self.bn1(self.conv1(x)))
        x = self.act2(self.bn2(self.conv2(x)))
        x = self.bn3(self.conv3(x))
        if self.downsample is not None:
            shortcut = self.downsample(shortcut)
        return self.act3(x + shortcut)


class ResNet(nn.Module):
    """timm ResNet; ``layers`` = [2,2,2,2] with BasicBlocks is resnet18."""

    def __init__(self, layers=(2, 2, 2, 2), in_chans: int = 3, block=BasicBlock):
        super().__init__()
        self.conv1 = nn.Conv2d(in_chans, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.act1 = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        inplanes = 64
        for i, (planes, n) in enumerate(zip((64, 128, 256, 512), layers)):
            stride = 1 if i == 0 else 2
            blocks = []
            for b in range(n):
                s = stride if b == 0 else 1
                ds = None
                if b == 0 and (s != 1 or inplanes != planes * block.expansion):
                    ds = nn.Sequential(nn.Conv2d(inplanes, planes * block.expansion, 1, stride=s, bias=False),
                                       nn.BatchNorm2d(planes * block.expansion))
                blocks.append(block(inplanes, planes, s, ds))
                inplanes = planes * block.expansion
            self.add_module(f'layer{i + 1}', nn.Sequential(*blocks))
        self.num_features = 512 * block.expansion
        # timm: global_pool + fc(Identity) for num_classes=0 -> no parameters.
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode='fan_out', nonlinearity='relu')

    def forward_features(self, x):
        x = self.maxpool(self.act1(self.bn1(self.conv1(x))))
        x = self.layer1(x)
        x = self.layer2(x)
        x = self.layer3(x)
        x = self.layer4(x)
        return x

    def forward(self, x):
        # timm forward_head with num_classes=0: global avg pool + flatten.
        return self.forward_features(x).mean(dim=(2, 3))


def create_model(model_name: str = 'resnet18', pretrained: bool = False, num_classes: int = 0, **kw):
    """Offline stand-in for ``timm.create_model`` (pretrained weights are a network
    fetch and unavailable here)."""
    depths = {'resnet18': (BasicBlock, (2, 2, 2, 2)), 'resnet34': (BasicBlock, (3, 4, 6, 3)),
              'resnet50': (Bottleneck, (3, 4, 6, 3)), 'resnet101': (Bottleneck, (3, 4, 23, 3)),
              'resnet152': (Bottleneck, (3, 8, 36, 3))}
    if model_name not in depths:
        raise ValueError(f'unsupported backbone {model_name!r}')
    assert num_classes == 0
    block, layers = depths[model_name]
    return ResNet(layers, block=block)


def make_head(num_features: int = 512) -> nn.Sequential:
    """inference_runner.py:36-48."""
    return nn.Sequential(
        nn.AdaptiveAvgPool2d(1),
        nn.Flatten(),
        nn.Linear(num_features, 512),
        nn.BatchNorm1d(512),
        nn.ReLU(),
        nn.Dropout(0.5),
        nn.Linear(512, 256),
        nn.BatchNorm1d(256),
        nn.ReLU(),
        nn.Dropout(0.3),
        nn.Linear(256, 2),
    )


class BinaryClassifier(nn.Module):
    """inference_runner.py:28-51: index 0 => Real, 1 => Synthetic."""

    def __init__(self, model_name: str = 'resnet18'):
        super().__init__()
        self.base = create_model(model_name, num_classes=0)
        self.head = make_head(self.base.num_features)

    def forward(self, x):
        return self.head(self.base.forward_features(x))


class ModularMultiHeadClassifier(nn.Module):
    """inference_runner.py:53-73: [B, N+1] = [syn_1..syn_N, mean(real_i)]."""

    def __init__(self, sub_models: List[nn.Module]):
        super().__init__()
        self.sub_models = nn.ModuleList(sub_models)

    def forward(self, x):
        real_list, syn_list = [], []
        for m in self.sub_models:
            out = m(x)
            real_list.append(out[:, 0:1])
            syn_list.append(out[:, 1:2])
        syn_cat = torch.cat(syn_list, dim=1)
        real_cat = torch.cat(real_list, dim=1)
        real_mean = torch.mean(real_cat, dim=1, keepdim=True)
        return torch.cat([syn_cat, real_mean], dim=1)


def per_head_logits(model: ModularMultiHeadClassifier, x: torch.Tensor) -> torch.Tensor:
    """[B, N, 2] raw per-head logits (what the HIP path gathers before merging)."""
    return torch.stack([m(x) for m in model.sub_models], dim=1)


def load_merged_state(sd: dict, backbone_name: str = 'resnet18') -> ModularMultiHeadClassifier:
    """Key mapping of inference_runner.py:88-117 (sorted integer sub-model indices,
    ``sub_models.<i>.<key>`` -> ``<key>``), strict: every key must be present."""
    idx = sorted({int(k.split('.')[1]) for k in sd if k.startswith('sub_models.') and k.split('.')[1].isdigit()})
    subs = []
    for i in idx:
        sm = BinaryClassifier(backbone_name)
        local = {k: sd[f'sub_models.{i}.{k}'] for k in sm.state_dict().keys()}
        sm.load_state_dict(local, strict=True)
        sm.eval()
        subs.append(sm)
    return ModularMultiHeadClassifier(subs).eval()
