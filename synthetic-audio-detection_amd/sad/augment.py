"""Host-side sampling of the trainer's random augmentation parameters.

The reference draws these inside ``SpectrogramDataset.__getitem__`` with torch's
global RNG (DataLoader workers): torchaudio ``FrequencyMasking(15)`` /
``TimeMasking(35)`` (``submodel_trainer.py:108-114,195-196``) and torchvision
``RandomResizedCrop(512, scale=(0.8, 1.0))`` (``:465-467``).  Only the integer
parameters are drawn here (same formulas, same RNG calls in the same order);
the masking, standardisation and crop-resize arithmetic run on the device
(``sad_specaug_norm_run`` / ``sad_crop_resize_run``).
"""
from __future__ import annotations

import math

import torch

FREQ_MASK_PARAM = 15
TIME_MASK_PARAM = 35
CROP_SCALE = (0.8, 1.0)
CROP_RATIO = (3.0 / 4.0, 4.0 / 3.0)


def mask_range(axis_len: int, mask_param: int, generator: torch.Generator | None = None):
    """torchaudio.functional.mask_along_axis (p = 1.0): returns the masked
    half-open index range [start, end) along one axis."""
    value = torch.rand(1, generator=generator) * mask_param
    min_value = torch.rand(1, generator=generator) * (axis_len - value)
    start = int(min_value.long().item())
    end = int((min_value.long() + value.long()).item())
    return start, end


def specaug_masks(n_mels: int = 128, n_frames: int = 251, generator: torch.Generator | None = None):
    """(f0, f1, t0, t1): FrequencyMasking then TimeMasking, as applied by the
    reference's nn.Sequential (frequency first)."""
    f0, f1 = mask_range(n_mels, FREQ_MASK_PARAM, generator)
    t0, t1 = mask_range(n_frames, TIME_MASK_PARAM, generator)
    return f0, f1, t0, t1


def random_resized_crop_params(height: int = 512, width: int = 512, scale=CROP_SCALE, ratio=CROP_RATIO,
                               generator: torch.Generator | None = None):
    """torchvision RandomResizedCrop.get_params -> (i, j, h, w)."""
    area = height * width
    log_ratio = torch.log(torch.tensor(ratio))
    for _ in range(10):
        target_area = area * torch.empty(1).uniform_(scale[0], scale[1], generator=generator).item()
        aspect_ratio = torch.exp(torch.empty(1).uniform_(log_ratio[0].item(), log_ratio[1].item(),
                                                         generator=generator)).item()
        w = int(round(math.sqrt(target_area * aspect_ratio)))
        h = int(round(math.sqrt(target_area / aspect_ratio)))
        if 0 < w <= width and 0 < h <= height:
            i = int(torch.randint(0, height - h + 1, size=(1,), generator=generator).item())
            j = int(torch.randint(0, width - w + 1, size=(1,), generator=generator).item())
            return i, j, h, w
    # fallback to the central crop
    in_ratio = float(width) / float(height)
    if in_ratio < min(ratio):
        w = width
        h = int(round(w / min(ratio)))
    elif in_ratio > max(ratio):
        h = height
        w = int(round(h * max(ratio)))
    else:
        w, h = width, height
    return (height - h) // 2, (width - w) // 2, h, w


FULL_IMAGE = (0, 0, 512, 512)
NO_MASK = (0, 0, 0, 0)
