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


def test_oracle_preprocess_waveform_mono_pad(tmp_path):
    """oracle preprocess_waveform (scipy WAV decode, torch mean, pad) on a stereo int16 file."""
    from oracle import audio as oaudio
    x = (np.random.RandomState(1).randn(2, 5000) * 1000).astype(np.int16)
    p = tmp_path / 's.wav'
    _write(p, x, 32000, 2)
    wf, sr = oaudio.preprocess_waveform(str(p))
    assert sr == 32000 and wf.shape == (128000,)
    assert torch.equal(wf[:5000], torch.from_numpy(x.astype(np.float32) / 32768.0).mean(0))
    assert torch.count_nonzero(wf[5000:]) == 0


def test_oracle_wav_decoders_agree(tmp_path):
    """scipy's WAV reader (oracle) and sad.audio.read_wav / load decode 8/16/24/32-bit alike."""
    from oracle import audio as oaudio
    rs = np.random.RandomState(5)
    cases = [(1, rs.randint(0, 256, (2, 300))), (2, rs.randint(-32768, 32768, (1, 300))),
             (3, rs.randint(-(1 << 23), 1 << 23, (2, 300))), (4, rs.randint(-(1 << 31), (1 << 31) - 1, (1, 300)))]
    for width, x in cases:
        p = tmp_path / f'w{width}.wav'
        _write(p, x, 22050, width)
        a, sra = audio.load(str(p))
        b, srb = oaudio.load(str(p))
        assert sra == srb == 22050 and a.shape == b.shape
        assert torch.equal(a, b), width
        raw, ch, sr = audio.read_wav(str(p))
        assert ch == x.shape[0] and sr == 22050 and raw.dtype == (np.int16 if width == 2 else np.float32)


RATES = [(44100, 32000), (48000, 32000), (16000, 32000), (22050, 32000), (8000, 32000), (96000, 32000)]


def test_oracle_resample_polyphase_vs_direct():
    """torchaudio's polyphase form (oracle.resample, fp32 conv1d) against the
    defining float64 sum (oracle.resample_direct): pins the polyphase index
    arithmetic that the HIP kernel shares; also the trainer's host resample."""
    from oracle import audio as oaudio
    rs = np.random.RandomState(2)
    for orig, new in RATES:
        x = (rs.randn(3001) * 0.3).astype(np.float32)
        ref = oaudio.resample_direct(x, orig, new)
        y = oaudio.resample(torch.from_numpy(x), orig, new).double().numpy()
        assert y.shape == ref.shape == (math.ceil(new * 3001 / orig),)
        # torchaudio forms the phase -p/new in fp32 (its arange / new), which moves
        # the taps by ~1e-5 against the exact float64 sum; an indexing error would be O(0.1)
        assert np.abs(y - ref).max() < 5e-5, (orig, new, np.abs(y - ref).max())
        h = audio.resample(torch.from_numpy(x), orig, new).double().numpy()
        assert np.array_equal(h, y), (orig, new)


def test_oracle_kernel_table_equals_host():
    from oracle import audio as oaudio
    for orig, new in RATES:
        g = math.gcd(orig, new)
        k1, w1 = oaudio._kernel(orig // g, new // g)
        k2, w2 = audio._sinc_resample_kernel(orig, new, g)
        assert w1 == w2 and torch.equal(k1, k2)


def test_window_starts_match_slice_waveform():
    import inference_runner as ir
    from sad import ingest
    cfg = ir.AudioConfig(overlap=0.85)
    for n in (128000, 128001, 140000, 500000, 127999):
        wf = torch.ones(n)
        chunks, ts = ir.slice_waveform(wf, 32000, cfg)
        window = int(cfg.window_size * 32000)
        starts = list(ingest.window_starts(n, window, int((1 - cfg.overlap) * window)))
        assert [s / 32000 for s in starts] == ts


def test_product_fbank_equals_torchaudio_restatement():
    """sad.audio.melscale_fbanks (the bank the device plan projects on, via
    sad_frontend_plan_create_fb) is the oracle's torchaudio restatement bit for
    bit, for the inference ('slaney') and trainer (None) banks -- and differs
    from the library's float64-rounded default bank (the reason it exists)."""
    import math

    import torch

    from oracle import frontend as ofe
    from sad.audio import melscale_fbanks
    for norm in ('slaney', None):
        a = melscale_fbanks(1025, 20.0, 12000.0, 128, 32000, norm == 'slaney')
        b = ofe.melscale_fbanks(1025, 20.0, 12000.0, 128, 32000, norm)
        assert a.dtype == torch.float32 and torch.equal(a, b)
    # the float64 evaluation of the same triangle, rounded once (what
    # sad_frontend_plan_create builds): bin 130 of mel 59 differs by 1e-5 relative
    hz2mel = lambda f: 2595.0 * math.log10(1.0 + f / 700.0)  # noqa: E731
    lo, hi = hz2mel(20.0), hz2mel(12000.0)
    pts = [700.0 * (10 ** ((lo + (hi - lo) * i / 129) / 2595.0) - 1.0) for i in range(130)]
    k, m = 130, 59
    f = 16000.0 * k / 1024
    v = max(0.0, min((f - pts[m]) / (pts[m + 1] - pts[m]), (pts[m + 2] - f) / (pts[m + 2] - pts[m + 1])))
    v *= 2.0 / (pts[m + 2] - pts[m])
    a = melscale_fbanks(1025, 20.0, 12000.0, 128, 32000, True)
    assert abs(float(a[k, m]) - v) > 1e-5 * v
