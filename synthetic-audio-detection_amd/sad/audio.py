"""Host-side audio ingestion: WAV decode and torchaudio-compatible resampling.

Replaces ``torchaudio.load`` and ``torchaudio.transforms.Resample`` as used by
``preprocess_waveform`` (inference_runner.py:144-155) and the trainer dataset
(submodel_trainer.py:143,150-153).  torchaudio is not available in this image;
these are restatements of its documented behaviour:

* ``load(path)`` -> (float32 [channels, frames], sample_rate), integer PCM
  scaled by 1/2^(bits-1) (torchaudio ``normalize=True``), float WAV as is.
  Supports RIFF/WAVE PCM 8/16/24/32-bit and IEEE float 32/64 (incl.
  WAVE_FORMAT_EXTENSIBLE).
* ``resample(wf, orig, new)`` -> torchaudio.functional.resample with its
  defaults (sinc_interp_hann, lowpass_filter_width=6, rolloff=0.99): windowed
  sinc kernel built in float64, cast to float32, applied as a strided conv1d.
  Used only by the trainer's Dataset, which runs in DataLoader worker
  processes on the host, as the reference's does (submodel_trainer.py:143-153).
  The inference path resamples on the device (sad.ingest, csrc/ingest.hip).
"""
from __future__ import annotations

import math
import struct

import numpy as np
import torch
import torch.nn.functional as F


def _read_chunks(data: bytes):
    if data[:4] != b'RIFF' or data[8:12] != b'WAVE':
        raise ValueError('not a RIFF/WAVE file')
    pos, fmt, payload = 12, None, None
    while pos + 8 <= len(data):
        cid, size = data[pos:pos + 4], struct.unpack('<I', data[pos + 4:pos + 8])[0]
        body = data[pos + 8:pos + 8 + size]
        if cid == b'fmt ':
            fmt = body
        elif cid == b'data':
            payload = body
        pos += 8 + size + (size & 1)
    if fmt is None or payload is None:
        raise ValueError('WAV file lacks fmt/data chunks')
    return fmt, payload


def _wav_layout(path: str):
    """RIFF walk over the chunk headers only -> (fmt bytes, data offset, data size)."""
    fmt = data_off = data_size = None
    with open(path, 'rb') as f:
        head = f.read(12)
        if len(head) < 12 or head[:4] != b'RIFF' or head[8:12] != b'WAVE':
            raise ValueError('not a RIFF/WAVE file')
        pos = 12
        while True:
            h = f.read(8)
            if len(h) < 8:
                break
            cid, size = h[:4], struct.unpack('<I', h[4:8])[0]
            if cid == b'fmt ':
                fmt = f.read(size)
            elif cid == b'data':
                data_off, data_size = pos + 8, size
            pos += 8 + size + (size & 1)
            f.seek(pos)
            if fmt is not None and data_off is not None:
                break
        end = f.seek(0, 2)
    if fmt is None or data_off is None:
        raise ValueError('WAV file lacks fmt/data chunks')
    return fmt, data_off, min(data_size, end - data_off)


def read_wav(path: str):
    """WAV -> (interleaved samples [frames * channels], channels, sample_rate).
    16-bit PCM stays int16 as stored (the device scales it, sad_pcm_mono_run),
    read straight from the file into one array; every other encoding is
    decoded to float32 with torchaudio.load's normalize=True scaling."""
    fmt, off, size = _wav_layout(path)
    tag, ch, sr, _, _, bits = struct.unpack('<HHIIHH', fmt[:16])
    if tag == 0xFFFE and len(fmt) >= 26:  # WAVE_FORMAT_EXTENSIBLE: sub-format GUID's first 2 bytes
        tag = struct.unpack('<H', fmt[24:26])[0]
    width = bits // 8
    n = size // (width * ch)
    if tag == 1 and bits == 16:
        return np.fromfile(path, '<i2', count=n * ch, offset=off), ch, sr
    with open(path, 'rb') as f:
        f.seek(off)
        raw = f.read(n * width * ch)
    if tag == 1:  # PCM
        if bits == 8:
            x = (np.frombuffer(raw, np.uint8).astype(np.float32) - 128.0) / 128.0
        elif bits == 24:
            b = np.frombuffer(raw, np.uint8).reshape(-1, 3).astype(np.int32)
            v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
            v = np.where(v >= 1 << 23, v - (1 << 24), v)
            x = v.astype(np.float32) / float(1 << 23)
        elif bits == 32:
            x = (np.frombuffer(raw, '<i4').astype(np.float64) / float(1 << 31)).astype(np.float32)
        else:
            raise ValueError(f'unsupported PCM width {bits}')
    elif tag == 3:  # IEEE float
        x = np.frombuffer(raw, '<f4' if bits == 32 else '<f8').astype(np.float32)
    else:
        raise ValueError(f'unsupported WAV format tag {tag:#x}')
    return x, ch, sr


def load(path: str):
    """torchaudio.load(path) for WAV files -> (Tensor[C, T] float32, sample_rate)."""
    x, ch, sr = read_wav(path)
    if x.dtype == np.int16:
        x = x.astype(np.float32) / 32768.0
    return torch.from_numpy(x.reshape(-1, ch).T.copy()), sr


def load_pcm16_mono(path: str):
    """Fast path for the common case (mono 16-bit PCM): (int16 ndarray [T], sr) or None."""
    with open(path, 'rb') as f:
        data = f.read()
    fmt, payload = _read_chunks(data)
    tag, ch, sr, _, _, bits = struct.unpack('<HHIIHH', fmt[:16])
    if tag != 1 or ch != 1 or bits != 16:
        return None
    return np.frombuffer(payload[:len(payload) // 2 * 2], '<i2').copy(), sr


def save_pcm16(path: str, pcm: np.ndarray, sr: int = 32000):
    import wave
    pcm = np.atleast_2d(pcm)
    with wave.open(path, 'wb') as w:
        w.setnchannels(pcm.shape[0])
        w.setsampwidth(2)
        w.setframerate(sr)
        w.writeframes(np.ascontiguousarray(pcm.T).astype('<i2').tobytes())


def melscale_fbanks(n_freqs: int, f_min: float, f_max: float, n_mels: int, sample_rate: int,
                    slaney: bool) -> torch.Tensor:
    """The mel filterbank [n_freqs, n_mels] exactly as torchaudio builds it for
    MelSpectrogram (inference_runner.py:158-166, norm='slaney'; trainer
    submodel_trainer.py:97-104, norm=None): htk mel points, triangles and the
    slaney area norm evaluated in torch fp32 arithmetic, op for op, so the
    weights are torchaudio's to the bit.  Plan-time data for
    sad_frontend_plan_create_fb (the device projects on these weights)."""
    hz = torch.linspace(0, sample_rate // 2, n_freqs, dtype=torch.float32)  # fp32 whatever the default dtype
    mel_lo = 2595.0 * math.log10(1.0 + f_min / 700.0)  # python float64 scalars
    mel_hi = 2595.0 * math.log10(1.0 + f_max / 700.0)
    pts = 700.0 * (10.0 ** (torch.linspace(mel_lo, mel_hi, n_mels + 2, dtype=torch.float32) / 2595.0) - 1.0)
    gaps = pts[1:] - pts[:-1]
    rel = pts.unsqueeze(0) - hz.unsqueeze(1)                 # [n_freqs, n_mels + 2]
    rising = (-1.0 * rel[:, :-2]) / gaps[:-1]
    falling = rel[:, 2:] / gaps[1:]
    fb = torch.max(torch.zeros(1), torch.min(rising, falling))
    if slaney:
        fb *= (2.0 / (pts[2:n_mels + 2] - pts[:n_mels])).unsqueeze(0)
    return fb


def _sinc_resample_kernel(orig: int, new: int, gcd: int, lowpass_filter_width: int = 6, rolloff: float = 0.99,
                          device=None):
    orig //= gcd
    new //= gcd
    base = min(orig, new) * rolloff
    width = math.ceil(lowpass_filter_width * orig / base)
    idx = torch.arange(-width, width + orig, dtype=torch.float64, device=device)[None, None] / orig
    t = torch.arange(0, -new, -1, device=device)[:, None, None] / new + idx
    t = t * base
    t = t.clamp_(-lowpass_filter_width, lowpass_filter_width)
    window = torch.cos(t * math.pi / lowpass_filter_width / 2) ** 2
    t = t * math.pi
    scale = base / orig
    kernels = torch.where(t == 0, torch.tensor(1.0).to(t), t.sin() / t)
    kernels = kernels * (window * scale)  # torchaudio: kernels *= window * scale
    return kernels.to(torch.float32), width


def resample(wf: torch.Tensor, orig_freq: int, new_freq: int) -> torch.Tensor:
    """torchaudio.functional.resample(wf, orig, new) with default arguments."""
    if orig_freq == new_freq:
        return wf
    gcd = math.gcd(int(orig_freq), int(new_freq))
    kernel, width = _sinc_resample_kernel(int(orig_freq), int(new_freq), gcd, device=wf.device)
    o, n = int(orig_freq) // gcd, int(new_freq) // gcd
    shape = wf.shape
    x = wf.reshape(-1, shape[-1])
    length = x.shape[1]
    x = F.pad(x, (width, width + o))
    y = F.conv1d(x[:, None], kernel, stride=o)
    y = y.transpose(1, 2).reshape(x.shape[0], -1)
    target = int(math.ceil(n * length / o))
    return y[..., :target].reshape(shape[:-1] + (-1,))
