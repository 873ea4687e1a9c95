"""Deterministic synthetic 4 s / 32 kHz int16 segments.

Counter-based hash PRNG (splitmix64 finaliser) keyed by (seed, segment, sample),
so any segment of a 1 M-segment shard can be regenerated independently and
bit-identically on the host (this module) and on the device
(``csrc/synth.hip``, exported as ``sad_synth_pcm``):

  noise  = floor((a+b+c+d - 131070) * 5675 / 65536)   a..d = 16-bit hash fields
           (Irwin-Hall(4) scaled to sigma ~ 0.1 FS = 3277 LSB, integer-only)
  tones  = sum_{i<k} amp_i * sin(2*pi*f_i*j/32000 + phi_i)    k in {1,2,3}
           f in [100, 11000) Hz, amp in [0.05, 0.30) FS, computed in float64
  pcm[j] = clip(noise + rint(tones), -32768, 32767)

The sinusoid term is float64 on both sides; libm ``sin`` may differ from the
device's by an ulp, which flips ``rint`` with negligible probability -- the
tests allow at most a handful of 1-LSB differences per million samples.
"""
from __future__ import annotations

import numpy as np

M64 = 0xFFFFFFFFFFFFFFFF
GOLD = 0x9E3779B97F4A7C15
GOLD2 = 0xD1B54A32D192ED03
SEG_SAMPLES = 128000
SAMPLE_RATE = 32000


def mix64(z):
    """splitmix64 finaliser on python ints or numpy uint64 arrays (wrapping)."""
    if isinstance(z, np.ndarray):
        z = z.astype(np.uint64, copy=True)
        z ^= z >> np.uint64(30)
        z *= np.uint64(0xBF58476D1CE4E5B9)
        z ^= z >> np.uint64(27)
        z *= np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
        return z
    z &= M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def segment_key(seed: int, seg: int) -> int:
    return mix64((mix64(seed & M64) + (seg * GOLD)) & M64)


def tone_params(seed: int, seg: int):
    """[(freq_hz, amp_lsb, phase_rad)] for one segment (1..3 tones)."""
    hs = mix64(segment_key(seed, seg) ^ 0x5EED5EED5EED5EED)
    k = 1 + (hs % 3)
    out = []
    for i in range(k):
        hi = mix64((hs + (i + 1) * GOLD2) & M64)
        f = 100.0 + ((hi & 0xFFFF) / 65536.0) * 10900.0
        amp = (0.05 + (((hi >> 16) & 0xFFFF) / 65536.0) * 0.25) * 32767.0
        ph = (((hi >> 32) & 0xFFFF) / 65536.0) * 2.0 * np.pi
        out.append((f, amp, ph))
    return out


def synth_segment(seed: int, seg: int, n: int = SEG_SAMPLES) -> np.ndarray:
    key = np.uint64(segment_key(seed, seg))
    j = np.arange(n, dtype=np.uint64)
    r = mix64(key + (j + np.uint64(1)) * np.uint64(GOLD2))
    a = (r & np.uint64(0xFFFF)).astype(np.int64)
    b = ((r >> np.uint64(16)) & np.uint64(0xFFFF)).astype(np.int64)
    c = ((r >> np.uint64(32)) & np.uint64(0xFFFF)).astype(np.int64)
    d = ((r >> np.uint64(48)) & np.uint64(0xFFFF)).astype(np.int64)
    noise = ((a + b + c + d - 131070) * 5675) >> 16
    jd = np.arange(n, dtype=np.float64)
    tones = np.zeros(n, dtype=np.float64)
    for f, amp, ph in tone_params(seed, seg):
        w = 2.0 * np.pi * f / float(SAMPLE_RATE)
        tones += amp * np.sin(w * jd + ph)
    x = noise + np.rint(tones).astype(np.int64)
    return np.clip(x, -32768, 32767).astype(np.int16)


def synth_labelled_clip(seed: int, idx: int, label: int, n: int = 2 * SEG_SAMPLES) -> np.ndarray:
    """Training clip with a learnable 2-class label:
    class 1 = white noise + a harmonic tone stack (fundamental 150-600 Hz,
    4 partials), class 0 = low-pass filtered noise (one-pole, a in [0.85, 0.97)).
    int16 [n] (default 8 s: the trainer's two 4 s segments)."""
    key = segment_key(seed ^ 0xC1A55, idx)
    j = np.arange(n, dtype=np.uint64)
    r = mix64(np.uint64(key) + (j + np.uint64(1)) * np.uint64(GOLD2))
    u = ((r >> np.uint64(11)).astype(np.float64)) / float(1 << 53) - 0.5
    h = mix64(key ^ 0xABCDEF)
    if label:
        f0 = 150.0 + (h & 0xFFFF) / 65536.0 * 450.0
        t = np.arange(n, dtype=np.float64) / SAMPLE_RATE
        x = 0.15 * u
        for k in range(1, 5):
            x += (0.2 / k) * np.sin(2.0 * np.pi * f0 * k * t + k)
    else:
        from scipy.signal import lfilter
        a = 0.85 + ((h >> 16) & 0xFFFF) / 65536.0 * 0.12
        x = lfilter([1.0 - a], [1.0, -a], u)
        x = 0.3 * x / max(1e-9, np.abs(x).max())
    return np.clip(np.rint(x * 32767.0), -32768, 32767).astype(np.int16)


def synth_batch(seed: int, first_seg: int, count: int, n: int = SEG_SAMPLES) -> np.ndarray:
    """[count, n] int16, segments first_seg .. first_seg+count-1."""
    return np.stack([synth_segment(seed, first_seg + i, n) for i in range(count)]) if count else \
        np.zeros((0, n), np.int16)
