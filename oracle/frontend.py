"""Oracle front end: waveform -> mel -> dB -> standardise -> resize (fp32, CPU).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restates, on plain torch, the third-party arithmetic that the reference calls at
``modular/source/inference_runner.py:157-174`` (``waveform_to_spectrogram``) and
``modular/source/submodel_trainer.py:97-105,191-203`` (trainer variant):

* torchaudio.transforms.MelSpectrogram  -> ``mel_spectrogram``
  (Spectrogram: periodic Hann(2048), hop 512, center=True, reflect pad,
  onesided, power 2 via ``abs().pow(2)``; MelScale: htk triangles, optional
  slaney area norm, ``(spec^T @ fb)^T``)
* torchaudio.transforms.AmplitudeToDB(top_db=80) -> ``amplitude_to_db``
* torchvision.transforms.Resize((512, 512)) on a [1,H,W] tensor ->
  ``resize_bilinear`` (bilinear, align_corners=False; antialias is a no-op for
  this upsample -- SURVEY.md 2.2)
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn.functional as F


@dataclass
class AudioConfig:
    """Mirror of ``inference_runner.py:127-132``."""
    sample_rate: int = 32000
    window_size: float = 4.0
    overlap: float = 0.85
    silence_threshold: float = 1e-4


@dataclass
class SpectrogramConfig:
    """Mirror of ``inference_runner.py:134-142``."""
    n_fft: int = 2048
    hop_length: int = 512
    n_mels: int = 128
    f_min: int = 20
    f_max: int = 12000
    top_db: int = 80
    norm: str = 'slaney'


# --- torchaudio.functional.melscale_fbanks (htk) -----------------------------
def _hz_to_mel_htk(freq: float) -> float:
    return 2595.0 * math.log10(1.0 + (freq / 700.0))


def _mel_to_hz_htk(mels: torch.Tensor) -> torch.Tensor:
    return 700.0 * (10.0 ** (mels / 2595.0) - 1.0)


def melscale_fbanks(n_freqs: int, f_min: float, f_max: float, n_mels: int,
                    sample_rate: int, norm: str | None = None) -> torch.Tensor:
    """fp32 [n_freqs, n_mels] filterbank, torchaudio ``melscale_fbanks`` semantics
    (called by MelScale at inference_runner.py:158-166 with norm='slaney',
    submodel_trainer.py:97-104 with norm=None)."""
    all_freqs = torch.linspace(0, sample_rate // 2, n_freqs)
    m_min = _hz_to_mel_htk(f_min)
    m_max = _hz_to_mel_htk(f_max)
    m_pts = torch.linspace(m_min, m_max, n_mels + 2)
    f_pts = _mel_to_hz_htk(m_pts)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts.unsqueeze(0) - all_freqs.unsqueeze(1)
    zero = torch.zeros(1)
    down_slopes = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up_slopes = slopes[:, 2:] / f_diff[1:]
    fb = torch.max(zero, torch.min(down_slopes, up_slopes))
    if norm is not None and norm == 'slaney':
        enorm = 2.0 / (f_pts[2:n_mels + 2] - f_pts[:n_mels])
        fb *= enorm.unsqueeze(0)
    return fb


def power_spectrogram(wf: torch.Tensor, n_fft: int = 2048, hop: int = 512) -> torch.Tensor:
    """torchaudio Spectrogram(power=2): [..., T] -> [..., n_fft//2+1, frames]
    (in wf's dtype: fp32 as the reference; float64 for the tests' exact values)."""
    shape = wf.shape
    w2 = wf.reshape(-1, shape[-1])
    window = torch.hann_window(n_fft, dtype=wf.dtype)
    spec = torch.stft(w2, n_fft=n_fft, hop_length=hop, win_length=n_fft, window=window,
                      center=True, pad_mode='reflect', normalized=False, onesided=True,
                      return_complex=True)
    spec = spec.reshape(shape[:-1] + spec.shape[-2:])
    return spec.abs().pow(2.0)


def mel_spectrogram(wf: torch.Tensor, sr: int = 32000, cfg: SpectrogramConfig | None = None,
                    norm: str | None = 'slaney') -> torch.Tensor:
    """MelSpectrogram: [..., T] -> [..., n_mels, frames] (fp32)."""
    cfg = cfg or SpectrogramConfig()
    spec = power_spectrogram(wf, cfg.n_fft, cfg.hop_length)
    fb = melscale_fbanks(cfg.n_fft // 2 + 1, float(cfg.f_min), float(cfg.f_max), cfg.n_mels, sr, norm)
    return torch.matmul(spec.transpose(-1, -2), fb.to(spec.dtype)).transpose(-1, -2)


def amplitude_to_db(x: torch.Tensor, top_db: float | None = 80.0) -> torch.Tensor:
    """torchaudio AmplitudeToDB(stype='power', top_db) (inference_runner.py:167,170).

    The top_db clamp is taken over the packed channel dims: for the reference's
    rank-3 [1, n_mels, frames] input that is the whole segment."""
    x_db = 10.0 * torch.log10(torch.clamp(x, min=1e-10))
    x_db -= 10.0 * 0.0  # db_multiplier = log10(max(amin, ref=1.0)) = 0
    if top_db is not None:
        shape = x_db.size()
        packed_channels = shape[-3] if x_db.dim() > 2 else 1
        x_db = x_db.reshape(-1, packed_channels, shape[-2], shape[-1])
        x_db = torch.max(x_db, (x_db.amax(dim=(-3, -2, -1)) - top_db).view(-1, 1, 1, 1))
        x_db = x_db.reshape(shape)
    return x_db


def resize_bilinear(x: torch.Tensor, size=(512, 512)) -> torch.Tensor:
    """torchvision Resize(size) on a [C,H,W] (or [N,C,H,W]) float tensor."""
    squeeze = x.dim() == 3
    if squeeze:
        x = x.unsqueeze(0)
    y = F.interpolate(x, size=size, mode='bilinear', align_corners=False, antialias=False)
    return y.squeeze(0) if squeeze else y


def standardize(spec: torch.Tensor) -> torch.Tensor:
    """inference_runner.py:171 -- (x - mean) / (std_unbiased + 1e-6)."""
    return (spec - spec.mean()) / (spec.std() + 1e-6)


def segment_map(wf: torch.Tensor, sr: int = 32000, cfg: SpectrogramConfig | None = None):
    """One 4 s window [T] -> (mel_db [1,128,251], standardised map [1,128,251]).

    This is inference_runner.py:169-171, i.e. the part of the front end the
    fused HIP kernel computes (resize is a separate, linear step)."""
    cfg = cfg or SpectrogramConfig()
    spec = mel_spectrogram(wf.unsqueeze(0), sr, cfg, norm=cfg.norm)
    spec_db = amplitude_to_db(spec, cfg.top_db)
    return spec_db, standardize(spec_db)


def waveform_to_spectrogram(waveform: torch.Tensor, sr: int, spec_cfg: SpectrogramConfig) -> torch.Tensor:
    """Restatement of inference_runner.py:157-174 -> [1,3,512,512]."""
    _, spec = segment_map(waveform, sr, spec_cfg)
    spec = resize_bilinear(spec, (512, 512))
    spec3 = spec.repeat(3, 1, 1)
    return spec3.unsqueeze(0)


def batch_maps(pcm_i16, sr: int = 32000, cfg: SpectrogramConfig | None = None, dtype=torch.float32):
    """[n, 128000] int16 (numpy or torch) -> (mel_db [n,128,251], std map [n,128,251]).

    Each segment goes through the reference's per-window path separately (the
    top-db clamp and the moments are per segment).
    dtype float64 runs the STFT, projection and dB arithmetic without fp32
    rounding; the filterbank stays torchaudio's fp32 bank (melscale_fbanks),
    only cast, as mel_spectrogram does with fb.to(spec.dtype)."""
    t = torch.as_tensor(pcm_i16)
    dbs, maps = [], []
    for i in range(t.shape[0]):
        wf = t[i].to(dtype) / 32768.0
        d, m = segment_map(wf, sr, cfg)
        dbs.append(d[0])
        maps.append(m[0])
    return torch.stack(dbs), torch.stack(maps)
