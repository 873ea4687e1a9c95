"""GPU: the device ingestion edge (csrc/ingest.hip, sad.ingest) against the oracle.

* sad_pcm_mono_run: int16 / fp32 interleaved -> mono fp32 + zero pad; bit-exact
  with torch's CPU mean (ATen: the channels summed in order, then sum / C, a
  true division) for 1-6 int16 channels and 1-4 fp32 channels; for 5-6 fp32
  channels ATen's CPU reduction sums in another order (within 2.5e-7);
* sad_resample_run: the impulse response IS the polyphase table (bit-exact with
  the oracle's float64 -> fp32 torchaudio kernel up to 1 fp32 ulp of cos/sin
  differences); random signals vs the oracle's torchaudio restatement (fp32
  conv1d) within 2e-6 absolute (fp32 sums of <= 459 taps in another order),
  incl. inputs shorter than the filter, a 1-sample input and the zero tail;
* sad_window_absmax_run: equal to torch's per-window max |x| (exact: max is
  order-free), NaN propagating;
* sad_frontend_run_windows: windows read in place give the same maps, bit for
  bit, as the same windows copied out;
* the drop-in preprocess_waveform on 44.1 kHz stereo / 48 kHz 24-bit files vs
  the oracle's (scipy decode, torch mean, torchaudio Resample restated); and
  main() on a long 44.1 kHz file vs the oracle pipeline's logits and labels.
"""
import json
import math
import wave

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'

RATES = [(44100, 32000), (48000, 32000), (16000, 32000), (22050, 32000), (8000, 32000), (96000, 32000),
         (32000, 44100)]


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


def test_pcm_mono_int16_and_f32():
    from sad import ingest
    rs = np.random.RandomState(0)
    for ch in (1, 2, 3, 4, 5, 6):
        x = rs.randint(-32768, 32768, size=(5003, ch)).astype(np.int16)
        ref = (torch.from_numpy(x.T.astype(np.float32)) / 32768.0).mean(dim=0)
        got = ingest.mono(torch.from_numpy(x.reshape(-1)).to(DEV), ch, 6000).cpu()
        assert got.shape == (6000,) and torch.count_nonzero(got[5003:]) == 0
        assert torch.equal(got[:5003], ref), ch
        xf = (rs.randn(777, ch) * 0.5).astype(np.float32)
        reff = torch.from_numpy(xf.T.copy()).mean(dim=0)
        gotf = ingest.mono(torch.from_numpy(xf.reshape(-1)).to(DEV), ch).cpu()
        assert gotf.shape == (777,)
        if ch <= 4:
            assert torch.equal(gotf, reff), ch
        else:
            assert (gotf - reff).abs().max() <= 2.5e-7


@pytest.mark.parametrize('orig,new', RATES)
def test_resample_impulse_is_the_kernel_table(orig, new):
    from oracle import audio as oaudio
    from sad import ingest
    g = math.gcd(orig, new)
    o, n = orig // g, new // g
    k, width = oaudio._kernel(o, n)
    k = k[:, 0, :]  # [new][K]
    K = k.shape[1]
    T = 4 * o + K + 7
    i0 = 2 * o + 3  # a unit impulse at sample i0
    x = torch.zeros(T)
    x[i0] = 1.0
    y = ingest.resampler(orig, new, DEV)(x.to(DEV)).cpu()
    # y[j*new + p] = kernel[p][i0 - j*o + width] wherever that tap exists
    exp = torch.zeros_like(y)
    for j in range(y.shape[0] // n + 1):
        kk = i0 - j * o + width
        if 0 <= kk < K:
            for p in range(n):
                m = j * n + p
                if m < y.shape[0]:
                    exp[m] = k[p, kk]
    ulp = torch.finfo(torch.float32).eps * exp.abs().clamp_min(1e-30)
    assert ((y - exp).abs() <= ulp).all(), (y - exp).abs().max().item()


@pytest.mark.parametrize('orig,new', RATES)
def test_resample_vs_oracle(orig, new):
    from oracle import audio as oaudio
    from sad import ingest
    rs = np.random.RandomState(orig % 97)
    for T in (1, 5, 37, 4410, 44100 + 17):
        x = (rs.randn(T) * 0.3).astype(np.float32)
        ref = oaudio.resample(torch.from_numpy(x), orig, new)
        r = ingest.resampler(orig, new, DEV)
        assert r.out_len(T) == ref.shape[0]
        y = r(torch.from_numpy(x).to(DEV), min_len=ref.shape[0] + 100).cpu()
        assert torch.count_nonzero(y[ref.shape[0]:]) == 0
        err = (y[:ref.shape[0]] - ref).abs().max().item() if T > 0 else 0.0
        assert err <= 2e-6, (orig, new, T, err)


def test_window_absmax_and_nan():
    from sad import ingest
    rs = np.random.RandomState(3)
    x = torch.from_numpy((rs.randn(400000) * 0.01).astype(np.float32))
    x[190000:200000] *= 1e-3
    x[333333] = -7.0
    window, hop = 128000, 19200
    nw = len(ingest.window_starts(x.shape[0], window, hop))
    got = ingest.window_absmax(x.to(DEV), window, hop, nw).cpu()
    ref = torch.stack([x[s:s + window].abs().max() for s in ingest.window_starts(x.shape[0], window, hop)])
    assert torch.equal(got, ref)
    x[150000] = float('nan')
    got = ingest.window_absmax(x.to(DEV), window, hop, nw).cpu()
    ref = torch.stack([x[s:s + window].abs().max() for s in ingest.window_starts(x.shape[0], window, hop)])
    assert torch.equal(torch.isnan(got), torch.isnan(ref))
    assert torch.equal(got[~torch.isnan(got)], ref[~torch.isnan(ref)])


def test_select_windows_matches_slice_waveform():
    import inference_runner as ir
    from sad import ingest
    rs = np.random.RandomState(4)
    x = torch.from_numpy((rs.randn(700000) * 0.05).astype(np.float32))
    x[128000:300000] *= 1e-4  # quiet stretch: some windows skipped
    for overlap in (0.0, 0.85):
        cfg = ir.AudioConfig(overlap=overlap, silence_threshold=1e-3)
        chunks, ts = ir.slice_waveform(x, 32000, cfg)
        starts, ts2 = ingest.select_windows(x.to(DEV), 32000, cfg.window_size, cfg.overlap, cfg.silence_threshold)
        assert ts2 == ts and len(starts) == len(chunks) < len(ingest.window_starts(700000, 128000,
                                                                                   int((1 - overlap) * 128000)))
        for s, c in zip(starts, chunks):
            assert torch.equal(x[s:s + 128000], c)


def test_frontend_windows_equal_copied_windows():
    from sad import engine, ingest
    rs = np.random.RandomState(6)
    x = torch.from_numpy((rs.randn(600000) * 0.1).astype(np.float32)).to(DEV)
    starts = [0, 19200, 38400, 100001, 200003, 600000 - 128000]  # odd starts: the scalar-load path
    fe = engine.FrontEnd(DEV)
    w = ingest.Windows(x, starts, 128000)
    m1, db1 = fe.windows(x, w.offsets, want_db=True)
    copies = torch.stack([x[s:s + 128000] for s in starts]).contiguous()
    m2, db2 = fe(copies, want_db=True)
    assert torch.equal(m1, m2) and torch.equal(db1, db2)


@pytest.mark.parametrize('sr,width,ch', [(44100, 2, 2), (48000, 3, 1), (32000, 2, 2), (16000, 1, 1)])
def test_preprocess_waveform_vs_oracle(tmp_path, sr, width, ch):
    import inference_runner as ir
    from oracle import audio as oaudio
    rs = np.random.RandomState(sr % 101)
    T = int(sr * 2.6)
    lim = {1: (0, 256), 2: (-32768, 32768), 3: (-(1 << 23), 1 << 23)}[width]
    x = rs.randint(lim[0], lim[1], size=(ch, T))
    p = tmp_path / f'in_{sr}_{width}_{ch}.wav'
    _write(p, x, sr, width)
    wf, sr2 = ir.preprocess_waveform(str(p), ir.AudioConfig(), DEV)
    ref, sr3 = oaudio.preprocess_waveform(str(p))
    assert sr2 == sr3 == 32000 and wf.shape == ref.shape == (128000,) and wf.is_cuda
    err = (wf.cpu() - ref).abs().max().item()
    if sr == 32000:
        assert err == 0.0
    else:
        assert err <= 2e-6, err


def test_main_long_resampled_file_vs_oracle(tmp_path):
    """main() on a 44.1 kHz stereo file of ~23 s (resample + 5 windows, one of them
    silent) against the oracle pipeline: decode -> mono -> resample -> slice ->
    per-window spectrogram -> the fixture model (fp32), same labels, logits
    within the 1e-3 north-star bar through the percentages."""
    import inference_runner as ir
    from conftest import merged_sd
    from oracle import audio as oaudio
    from oracle import decision as odec
    from oracle import frontend as ofe
    from oracle import resnet as ores
    sd = merged_sd('n6')
    names = [f'Synthetic{chr(65 + i)}' for i in range(6)] + ['Real']
    mp = tmp_path / 'm.pth'
    torch.save({'state_dict': sd, 'metadata': {'class_names': names}}, mp)
    rs = np.random.RandomState(8)
    sr = 44100
    T = int(sr * 22.9)
    t = np.arange(T) / sr
    sig = 0.3 * np.sin(2 * np.pi * (300 + 900 * t / t[-1]) * t) + 0.05 * rs.randn(T)
    sig[int(sr * 8.2):int(sr * 12.5)] *= 1e-4  # a silent window (at main()'s threshold 1e-3)
    x = np.stack([sig, np.roll(sig, 37)]) * 20000
    p = tmp_path / 'long.wav'
    _write(p, x.astype(np.int16), sr, 2)
    out = tmp_path / 'o.json'
    js = ir.main(['--merged-model', str(mp), '--audio', str(p), '--output-json', str(out)])
    # oracle
    wf, _ = oaudio.preprocess_waveform(str(p))
    cfg = ir.AudioConfig(sample_rate=32000, window_size=4.0, overlap=0.0, silence_threshold=1e-3)
    chunks, ts = odec.slice_waveform(wf, 32000, cfg)
    assert len(chunks) == len(js['segments']) >= 3
    assert [s['start_sec'] for s in js['segments']] == ts
    model = ores.load_merged_state(sd)
    with torch.no_grad():
        specs = torch.cat([ofe.waveform_to_spectrogram(c, 32000, ofe.SpectrogramConfig()) for c in chunks])
        logits = model(specs)
    labels = [odec.interpret_multihead_logits(r, 0.5, names[:-1], names[-1])[0] for r in logits]
    assert [s['label'] for s in js['segments']] == labels
    probs = torch.sigmoid(logits).mean(0).numpy() * 100
    got = [js['percentages'][k] for k in names]
    assert np.abs(np.array(got) - probs).max() <= 1e-3 * 25, (got, probs)  # |dp| <= |dlogit| / 4
    assert json.load(open(out)) == js


@pytest.mark.parametrize('sr,frames', [(44100, 0), (44100, 1), (48000, 3), (32000, 0)])
def test_preprocess_tiny_files_vs_oracle(tmp_path, sr, frames):
    """Empty and few-sample files: the resampler's zero-length / shorter-than-
    the-filter paths, then the zero pad to one window."""
    import inference_runner as ir
    from oracle import audio as oaudio
    x = np.array([[12000, -7000, 300][:frames]] * 2, dtype=np.int64).reshape(2, frames)
    p = tmp_path / f'tiny_{sr}_{frames}.wav'
    _write(p, x, sr, 2)
    wf, _ = ir.preprocess_waveform(str(p), ir.AudioConfig(), DEV)
    if frames == 0 and sr != 32000:
        # torchaudio's resample views an empty waveform as [-1, 0] and raises, so the
        # reference's preprocess_waveform fails on such a file; the device path
        # returns the zero window (and main() then writes the empty-result JSON)
        with pytest.raises(RuntimeError):
            oaudio.preprocess_waveform(str(p))
        assert wf.shape == (128000,) and torch.count_nonzero(wf) == 0
        return
    ref, _ = oaudio.preprocess_waveform(str(p))
    assert wf.shape == ref.shape == (128000,)
    assert (wf.cpu() - ref).abs().max().item() <= 2e-6


def test_main_empty_resampled_file(tmp_path):
    import inference_runner as ir
    from conftest import merged_sd
    mp = tmp_path / 'm.pth'
    torch.save({'state_dict': merged_sd('n2'), 'metadata': {'class_names': ['A', 'B', 'Real']}}, mp)
    p = tmp_path / 'empty.wav'
    _write(p, np.zeros((2, 0), np.int64), 44100, 2)
    out = tmp_path / 'o.json'
    js = ir.main(['--merged-model', str(mp), '--audio', str(p), '--output-json', str(out)])
    assert js == {'filename': str(p), 'segments': [], 'percentages': {}}


def test_select_windows_edges():
    """slice_waveform's edge behaviour on the device path: overlap 1.0 gives a
    zero hop (range() refuses it, so ValueError), a waveform shorter than one
    window gives no windows, exactly one window gives one."""
    from sad import ingest
    x = torch.full((128000,), 0.5, device=DEV)
    with pytest.raises(ValueError):
        ingest.select_windows(x, 32000, 4.0, 1.0, 1e-3)
    assert ingest.select_windows(x[:127999].contiguous(), 32000, 4.0, 0.0, 1e-3) == ([], [])
    assert ingest.select_windows(x, 32000, 4.0, 0.85, 1e-3) == ([0], [0.0])
    with pytest.raises(ValueError):
        ingest.Windows(x, [1], 128000)  # past the end
