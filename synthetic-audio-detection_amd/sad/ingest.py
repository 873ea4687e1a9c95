"""Device-side ingestion of long audio files.

The reference's ``preprocess_waveform`` + ``slice_waveform`` + per-window
``waveform_to_spectrogram`` (inference_runner.py:144-190, 276-289) turn one WAV
into a list of 4 s host tensors.  Here the file's samples go to HBM once, as
stored (int16, or host-decoded fp32 for other encodings), and the rest runs on
libsad (csrc/ingest.hip, include/sad.h "ingestion"):

  load_waveform   interleaved PCM -> mono fp32 -> (resample to 32 kHz) -> pad
  select_windows  window starts at the reference's hop; the silence test on the
                  device (max |x| per window); the host sees one float per window
  Windows         the kept windows' start offsets on the device, read in place
                  by the front end (sad_frontend_run_windows)

The host work left is the WAV header parse and the keep/skip decision over the
per-window maxima (the same fp32 comparison as ``piece.abs().max() < thr``).
"""
from __future__ import annotations

import ctypes
from typing import List, Tuple

import numpy as np
import torch

from . import _lib
from . import audio as _audio


def _dev(device) -> torch.device:
    d = torch.device(device)
    if d.type != 'cuda':
        raise RuntimeError(f'libsad runs on an MI355X only (device={device!r}); there is no CPU path')
    return d if d.index is not None else torch.device('cuda', torch.cuda.current_device())


class Resampler:
    """torchaudio.transforms.Resample(orig_freq, new_freq) (sinc_interp_hann,
    width 6, rolloff 0.99) on the device: inference_runner.py:148."""

    def __init__(self, orig_freq: int, new_freq: int, device='cuda'):
        self.device = _dev(device)
        self.orig_freq, self.new_freq = int(orig_freq), int(new_freq)
        self._plan = _lib.P()
        with torch.cuda.device(self.device):
            _lib.call('sad_resample_plan_create', self.orig_freq, self.new_freq, ctypes.byref(self._plan))

    def out_len(self, n_in: int) -> int:
        n = _lib.I64()
        _lib.call('sad_resample_out_len', self._plan, int(n_in), ctypes.byref(n))
        return n.value

    def __call__(self, x: torch.Tensor, min_len: int = 0) -> torch.Tensor:
        """x [T] fp32 on the device -> [max(ceil(new*T/orig), min_len)] (zero tail)."""
        assert x.dtype == torch.float32 and x.dim() == 1 and x.is_contiguous() and x.device == self.device
        n_out = self.out_len(x.shape[0])
        y = torch.empty(max(n_out, int(min_len)), device=self.device, dtype=torch.float32)
        with torch.cuda.device(self.device):
            _lib.call('sad_resample_run', self._plan, _lib.ptr(x), x.shape[0], _lib.ptr(y), y.shape[0],
                      _lib.stream_handle(self.device))
        return y

    def __del__(self):
        try:
            if getattr(self, '_plan', None):
                _lib.load().sad_resample_plan_destroy(self._plan)
        except Exception:
            pass


_RESAMPLERS = {}


def resampler(orig_freq: int, new_freq: int, device='cuda') -> Resampler:
    d = _dev(device)
    key = (int(orig_freq), int(new_freq), str(d))
    if key not in _RESAMPLERS:
        _RESAMPLERS[key] = Resampler(orig_freq, new_freq, d)
    return _RESAMPLERS[key]


def mono(pcm: torch.Tensor, channels: int, out_len: int = 0) -> torch.Tensor:
    """Interleaved [frames * channels] int16 / fp32 on the device -> mono fp32
    [max(frames, out_len)]: torchaudio.load scaling + waveform.mean(dim=0) + zero pad."""
    assert pcm.dim() == 1 and pcm.is_contiguous() and pcm.dtype in (torch.int16, torch.float32)
    frames = pcm.shape[0] // channels
    dev = pcm.device
    out = torch.empty(max(frames, int(out_len)), device=dev, dtype=torch.float32)
    fmt = _lib.SAD_PCM_I16 if pcm.dtype == torch.int16 else _lib.SAD_PCM_F32
    with torch.cuda.device(dev):
        _lib.call('sad_pcm_mono_run', _lib.ptr(pcm), fmt, frames, int(channels), _lib.ptr(out), out.shape[0],
                  _lib.stream_handle(dev))
    return out


def waveform_from_samples(samples: np.ndarray, channels: int, sr: int, target_sr: int = 32000,
                          min_len: int = 0, device='cuda') -> Tuple[torch.Tensor, int]:
    """preprocess_waveform (inference_runner.py:144-155) from decoded WAV
    samples: upload as stored, mono, resample when sr != target_sr, zero-pad
    to min_len samples (the window) -> (fp32 [T] on the device, target_sr)."""
    dev = _dev(device)
    if samples.dtype not in (np.int16, np.float32):
        samples = samples.astype(np.float32)
    pcm = torch.from_numpy(np.ascontiguousarray(samples.reshape(-1))).to(dev)
    if int(sr) == int(target_sr):
        return mono(pcm, channels, min_len), int(sr)
    wf = mono(pcm, channels)
    return resampler(sr, target_sr, dev)(wf, min_len), int(target_sr)


def load_waveform(path: str, target_sr: int = 32000, min_len: int = 0, device='cuda') -> Tuple[torch.Tensor, int]:
    """WAV file -> (mono fp32 [T] at target_sr on the device, target_sr)."""
    samples, ch, sr = _audio.read_wav(path)
    return waveform_from_samples(samples, ch, sr, target_sr, min_len, device)


def window_absmax(wf: torch.Tensor, window: int, hop: int, n_windows: int) -> torch.Tensor:
    """max |wf[w*hop : w*hop + window]| for w < n_windows (device fp32 [n_windows])."""
    assert wf.dtype == torch.float32 and wf.dim() == 1 and wf.is_contiguous()
    out = torch.empty(max(int(n_windows), 0), device=wf.device, dtype=torch.float32)
    with torch.cuda.device(wf.device):
        _lib.call('sad_window_absmax_run', _lib.ptr(wf), wf.shape[0], int(window), int(hop), int(n_windows),
                  _lib.ptr(out), _lib.stream_handle(wf.device))
    return out


def window_starts(n: int, window: int, hop: int) -> range:
    """slice_waveform's start indices: range(0, n - window + 1, hop) (inference_runner.py:180)."""
    return range(0, n - window + 1, hop)


def select_windows(wf: torch.Tensor, sr: int, window_size: float, overlap: float,
                   silence_threshold: float) -> Tuple[List[int], List[float]]:
    """slice_waveform (inference_runner.py:176-190) on a device waveform: the
    kept windows' start samples and start times (s).  A window is skipped when
    its max |x| < silence_threshold, compared in fp32 as torch compares a
    float32 tensor with a Python float."""
    window = int(window_size * sr)
    hop = int((1 - overlap) * window)
    if hop <= 0:
        raise ValueError(f'hop of {hop} samples (overlap={overlap}): range() would reject it too')
    starts = window_starts(wf.shape[0], window, hop)
    if len(starts) == 0:
        return [], []
    mx = window_absmax(wf, window, hop, len(starts)).cpu().numpy()
    keep = ~(mx < np.float32(silence_threshold))
    kept = [s for s, k in zip(starts, keep) if k]
    return kept, [s / sr for s in kept]


class Windows:
    """The kept windows of one device waveform: the waveform, the window length
    and the start offsets (int64, on the device) that the front end reads
    them at."""

    def __init__(self, wf: torch.Tensor, starts: List[int], window: int):
        self.wf, self.window = wf, int(window)
        self.starts = list(starts)
        if any(s < 0 or s + self.window > wf.shape[0] for s in self.starts):
            raise ValueError('window start out of range')
        self.offsets = torch.tensor(self.starts, dtype=torch.int64).to(wf.device)

    def __len__(self):
        return len(self.starts)
