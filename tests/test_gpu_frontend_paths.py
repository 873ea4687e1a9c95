"""Front end (fe_mel_db_kernel, csrc/frontend.hip): the int16 paths around the
PCM prefetch give the same maps as the paths that do not prefetch.

* an odd segment stride turns the aligned pair loads (and the prefetch) off:
  the strided segments must match their contiguous copies bit for bit;
* int16 PCM against the same samples as fp32 / 32768 (the float path never
  prefetches; the int16 window carries the exact power-of-two scale), for the
  default plan, an odd hop (pairs off) and a segment shorter than one frame's
  FFT (2,048 samples: the prefetch reads a stand-in buffer, never used).

Reference behaviour: torchaudio MelSpectrogram(center=True, reflect) +
AmplitudeToDB(top_db=80) + standardisation, inference_runner.py:157-171; the
values themselves are pinned against the oracle by test_gpu_parity.py."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda', 0)


def _pcm(n_seg, n, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return (torch.randn(n_seg, n, device=DEV, generator=g) * 6000).clamp(-32768, 32767).to(torch.int16)


def test_int16_odd_stride_equals_contiguous():
    from sad import engine
    fe = engine.FrontEnd(DEV)
    n, B = fe.n_samples, 5
    base = _pcm(1, B * (n + 1), 11)[0]
    strided = base.view(B, n + 1)[:, :n]  # row stride n + 1 (odd)
    assert strided.stride(0) % 2 == 1
    m1, db1 = fe(strided, want_db=True)
    m2, db2 = fe(strided.contiguous(), want_db=True)
    assert torch.equal(m1, m2) and torch.equal(db1, db2)


@pytest.mark.parametrize('kw', [{}, {'hop': 511}, {'n_samples': 1500}], ids=['default', 'odd-hop', 'short'])
def test_int16_equals_f32(kw):
    from sad import engine
    fe = engine.FrontEnd(DEV, **kw)
    pcm = _pcm(4, fe.n_samples, 12)
    m16, db16 = fe(pcm, want_db=True)
    m32, db32 = fe(pcm.float() / 32768.0, want_db=True)
    assert torch.isfinite(m16).all()
    assert torch.equal(m16, m32) and torch.equal(db16, db32)
