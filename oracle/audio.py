"""Oracle ingestion: WAV -> mono fp32 -> torchaudio Resample -> pad (CPU).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restates ``preprocess_waveform`` (``modular/source/inference_runner.py:144-155``)
and the third-party calls in it:

* ``torchaudio.load(path)`` (normalize=True) -> ``load``: decoded by scipy's
  independent WAV reader (``scipy.io.wavfile``), integer PCM scaled by
  1/2^(bits-1) (8-bit: (x - 128) / 128), float as stored;
* ``waveform.mean(dim=0)`` -> torch's own mean on the [C, T] tensor;
* ``torchaudio.transforms.Resample(sr, 32000)`` (sinc_interp_hann,
  lowpass_filter_width 6, rolloff 0.99) -> ``resample``, torchaudio's
  polyphase form (float64 kernel built by ``_get_sinc_resample_kernel``,
  rounded to fp32, ``F.conv1d`` with stride orig) restated on torch;
  ``resample_direct`` evaluates the same band-limited interpolation in float64
  from its defining sum, y[m] = sum_i x[i] h(i/orig - m/new), with no polyphase
  index arithmetic: the cross-check of the polyphase indexing.

torchaudio is absent here, so bit-identity with a torchaudio build is
unpinned; the kernel formula follows torchaudio's published source
(functional.py ``_get_sinc_resample_kernel`` / ``_apply_sinc_resample_kernel``,
torchaudio 2.x), including its fp32 ``arange(0, -new, -1) / new``.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F


def load(path: str):
    """torchaudio.load(path) -> (float32 [C, T], sr) via scipy.io.wavfile."""
    from scipy.io import wavfile
    sr, data = wavfile.read(path)
    data = np.atleast_2d(data.T) if data.ndim == 2 else data[None, :]
    if data.dtype == np.uint8:
        x = (data.astype(np.float32) - 128.0) / 128.0
    elif data.dtype == np.int16:
        x = data.astype(np.float32) / 32768.0
    elif data.dtype == np.int32:  # 32-bit PCM, and 24-bit PCM left-justified by scipy
        x = (data.astype(np.float64) / float(1 << 31)).astype(np.float32)
    else:
        x = data.astype(np.float32)
    return torch.from_numpy(np.ascontiguousarray(x)), int(sr)


def _kernel(orig: int, new: int, lowpass_filter_width: int = 6, rolloff: float = 0.99):
    """torchaudio _get_sinc_resample_kernel (orig, new already reduced by the gcd)."""
    base = min(orig, new) * rolloff
    width = math.ceil(lowpass_filter_width * orig / base)
    idx = torch.arange(-width, width + orig, dtype=torch.float64)[None, None] / orig
    t = torch.arange(0, -new, -1)[:, None, None] / new + idx  # int / int: fp32, promoted by the add
    t = t * base
    t = t.clamp(-lowpass_filter_width, lowpass_filter_width)
    window = torch.cos(t * math.pi / lowpass_filter_width / 2) ** 2
    t = t * math.pi
    scale = base / orig
    kernels = torch.where(t == 0, torch.tensor(1.0, dtype=torch.float64), t.sin() / t)
    kernels = kernels * (window * scale)
    return kernels.to(torch.float32), width


def resample(wf: torch.Tensor, orig_freq: int, new_freq: int) -> torch.Tensor:
    """torchaudio.functional.resample(wf, orig_freq, new_freq), fp32 [..., T]."""
    if orig_freq == new_freq:
        return wf
    g = math.gcd(int(orig_freq), int(new_freq))
    o, n = int(orig_freq) // g, int(new_freq) // g
    kernel, width = _kernel(o, n)
    shape = wf.shape
    x = wf.reshape(-1, shape[-1])
    length = x.shape[1]
    x = F.pad(x, (width, width + o))
    y = F.conv1d(x[:, None], kernel, stride=o)
    y = y.transpose(1, 2).reshape(x.shape[0], -1)
    target = int(math.ceil(n * length / o))
    return y[..., :target].reshape(shape[:-1] + (-1,))


def resample_direct(x: np.ndarray, orig_freq: int, new_freq: int, lowpass_filter_width: int = 6,
                    rolloff: float = 0.99) -> np.ndarray:
    """float64 y[m] = sum_i x[i] h(i/orig - m/new), h(tau) = sinc(pi b tau) cos^2(pi b tau / 12) b/orig
    for |b tau| <= 6 (b = min(orig, new) * rolloff, rates reduced by the gcd),
    m < ceil(new * T / orig).  x: float [T]."""
    g = math.gcd(int(orig_freq), int(new_freq))
    o, n = int(orig_freq) // g, int(new_freq) // g
    b = min(o, n) * rolloff
    lpw = lowpass_filter_width
    T = x.shape[0]
    M = int(math.ceil(n * T / o))
    x = np.asarray(x, np.float64)
    y = np.zeros(M)
    reach = lpw * o / b  # input samples on either side of an output
    for m in range(M):
        c = m * o / n  # output m's position in input samples
        i0, i1 = max(0, math.ceil(c - reach)), min(T - 1, math.floor(c + reach))
        if i1 < i0:
            continue
        i = np.arange(i0, i1 + 1)
        tau = (i / o - m / n) * b
        tau = np.clip(tau, -lpw, lpw)
        w = np.cos(tau * math.pi / lpw / 2) ** 2
        s = np.where(tau == 0, 1.0, np.sin(np.pi * tau) / np.where(tau == 0, 1.0, np.pi * tau))
        y[m] = np.dot(x[i0:i1 + 1], s * w * (b / o))
    return y


def preprocess_waveform(path: str, sample_rate: int = 32000, window_size: float = 4.0):
    """inference_runner.py:144-155 -> (mono fp32 [T], sr) on the CPU."""
    wf, sr = load(path)
    wf = wf.mean(dim=0)
    if sr != sample_rate:
        wf = resample(wf, sr, sample_rate)
        sr = sample_rate
    needed = int(window_size * sr)
    if wf.shape[0] < needed:
        temp = torch.zeros(needed)
        temp[:wf.shape[0]] = wf
        wf = temp
    return wf, sr
