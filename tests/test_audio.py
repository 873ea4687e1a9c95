"""CPU: WAV ingestion and torchaudio-compatible resampling (sad.audio), and the
drop-in preprocess_waveform (inference_runner.py:144-155)."""
import math
import wave

import numpy as np
import torch

from sad import audio


def _write(path, data, sr, width):
    with wave.open(str(path), 'wb') as w:
        w.setnchannels(data.shape[0])
        w.setsampwidth(width)
        w.setframerate(sr)
        if width == 3:
            v = data.T.astype(np.int32).reshape(-1)
            b = np.stack([v & 255, (v >> 8) & 255, (v >> 16) & 255], 1).astype(np.uint8)
            w.writeframes(b.tobytes())
        else:
            w.writeframes(data.T.astype({1: np.uint8, 2: '<i2', 4: '<i4'}[width]).tobytes())


def test_wav_pcm16_stereo_roundtrip(tmp_path):
    x = (np.random.RandomState(0).randn(2, 1000) * 3000).astype(np.int16)
    p = tmp_path / 'a.wav'
    _write(p, x, 32000, 2)
    wf, sr = audio.load(str(p))
    assert sr == 32000 and wf.shape == (2, 1000) and wf.dtype == torch.float32
    assert torch.equal(wf, torch.from_numpy(x.astype(np.float32) / 32768.0))


def test_wav_pcm24_and_8(tmp_path):
    x = np.array([[-(1 << 23), -1, 0, 1, (1 << 23) - 1]])
    p = tmp_path / 'b.wav'
    _write(p, x, 16000, 3)
    wf, _ = audio.load(str(p))
    assert np.allclose(wf.numpy(), x / float(1 << 23))
    y = np.array([[0, 128, 255]])
    _write(tmp_path / 'c.wav', y, 8000, 1)
    wf, _ = audio.load(str(tmp_path / 'c.wav'))
    assert np.allclose(wf.numpy(), (y - 128) / 128.0)


def test_resample_identity_and_length():
    x = torch.randn(1, 44100)
    assert audio.resample(x, 32000, 32000) is x
    y = audio.resample(x, 44100, 32000)
    assert y.shape == (1, math.ceil(32000 * 44100 / 44100))


def test_resample_preserves_inband_tone():
    sr0, sr1, f = 48000, 32000, 1000.0
    t = np.arange(48000) / sr0
    x = torch.from_numpy(np.sin(2 * np.pi * f * t).astype(np.float32))
    y = audio.resample(x, sr0, sr1).numpy()
    ref = np.sin(2 * np.pi * f * np.arange(len(y)) / sr1)
    mid = slice(200, len(y) - 200)
    assert np.abs(y[mid] - ref[mid]).max() < 2e-3


def test_resample_kernel_matches_torchaudio_formula():
    """Known values of torchaudio's sinc_interp_hann kernel: centre tap of the
    phase-0 filter is rolloff * min/orig (scale), taps are symmetric."""
    k, width = audio._sinc_resample_kernel(2, 1, 1)
    assert width == math.ceil(6 * 2 / 0.99)
    k = k[0, 0].double()
    centre = k[width].item()
    assert abs(centre - 0.99 * 1 / 2) < 1e-6
    assert torch.allclose(k[width - 3], k[width + 3], atol=1e-7)


def test_preprocess_waveform_mono_pad(tmp_path):
    import inference_runner as ir
    x = (np.random.RandomState(1).randn(2, 5000) * 1000).astype(np.int16)
    p = tmp_path / 's.wav'
    _write(p, x, 32000, 2)
    wf, sr = ir.preprocess_waveform(str(p), ir.AudioConfig())
    assert sr == 32000 and wf.shape == (128000,)
    assert torch.equal(wf[:5000], torch.from_numpy(x.astype(np.float32) / 32768.0).mean(0))
    assert torch.count_nonzero(wf[5000:]) == 0
