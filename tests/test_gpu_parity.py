"""GPU parity: libsad (HIP, gfx950) against the golden fixtures and the CPU oracle.

Tolerances (north_star: |dlogit| <= 1e-3 fp32, bit-exact indexing/argmax):
  * front end, fp32:  dB map |d| <= 2e-3 dB, standardised map |d| <= 2e-4
  * stem / backbone features, fp32 mode: relative to the oracle <= 1e-4
  * logits, fp32 mode: |d| <= 1e-3 against the reference-generated fixtures
  * decisions: identical labels to the reference's interpret_multihead_logits
  * bf16 throughput mode: logits |d| <= 1e-1 (reported, not the parity gate)
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import merged_sd

pytestmark = pytest.mark.gpu

DEV = 'cuda:0'


@pytest.fixture(scope='module')
def fe():
    from sad.engine import FrontEnd
    return FrontEnd(DEV)


def test_frontend_matches_golden(fe, golden_frontend):
    pcm = torch.from_numpy(golden_frontend['pcm']).to(DEV)
    m, db = fe(pcm, want_db=True)
    torch.cuda.synchronize()
    ddb = (db.cpu() - torch.from_numpy(golden_frontend['mel_db'])).abs().max().item()
    dm = (m.cpu() - torch.from_numpy(golden_frontend['std_map'])).abs().max().item()
    print(f'frontend max|d dB| = {ddb:.3e}, max|d map| = {dm:.3e}')
    assert ddb <= 2e-3
    assert dm <= 2e-4


def test_frontend_batch_vs_oracle(fe):
    """configs[1]: a 1,024-segment batch through the device synth + front end,
    EVERY segment checked against the oracle (torch.stft path; ~2 s of CPU)."""
    from oracle import frontend as ofe
    from sad import _lib
    n = 1024
    pcm = torch.empty(n, 128000, dtype=torch.int16, device=DEV)
    _lib.call('sad_synth_pcm', 11, 0, n, 128000, _lib.ptr(pcm), _lib.stream_handle(torch.device(DEV)))
    m = fe(pcm)
    torch.cuda.synchronize()
    host, dev_maps, d = pcm.cpu(), m.cpu(), 0.0
    for s in range(0, n, 128):
        _, ref = ofe.batch_maps(host[s:s + 128])
        d = max(d, (dev_maps[s:s + 128] - ref).abs().max().item())
    print(f'frontend batch1024 (all segments) max|d map| = {d:.3e}')
    assert d <= 2e-4
    assert torch.isfinite(m).all()


def test_synth_device_matches_host():
    from sad import _lib
    from sad.synth import synth_batch
    pcm = torch.empty(3, 128000, dtype=torch.int16, device=DEV)
    _lib.call('sad_synth_pcm', 5, 100, 3, 128000, _lib.ptr(pcm), _lib.stream_handle(torch.device(DEV)))
    host = torch.from_numpy(synth_batch(5, 100, 3))
    diff = (pcm.cpu().to(torch.int32) - host.to(torch.int32)).abs()
    assert diff.max().item() <= 1 and (diff > 0).sum().item() <= 3


def test_resize_matches_oracle(golden_frontend):
    from oracle import frontend as ofe
    from sad.engine import resize
    m = torch.from_numpy(golden_frontend['std_map']).to(DEV)
    img = resize(m)
    ref = ofe.resize_bilinear(torch.from_numpy(golden_frontend['std_map']).unsqueeze(1), (512, 512))[:, 0]
    assert (img.cpu() - ref).abs().max().item() <= 1e-5
    rows = img.double().sum(2).cpu().numpy()
    assert np.abs(rows - golden_frontend['img_rowsum']).max() <= 1e-3


def _oracle_sub(tag, i=0):
    from oracle import resnet as ores
    return ores.load_merged_state(merged_sd(tag)).sub_models[i]


def test_stem_fp32_vs_oracle(golden_frontend):
    from oracle import frontend as ofe
    from sad.engine import Backbone, split_merged_state
    sd = merged_sd('n6')
    _, bases, _ = split_merged_state(sd)
    bb = Backbone(bases[0], DEV, 'fp32')
    maps = torch.from_numpy(golden_frontend['std_map'])
    out = bb.stem(maps.to(DEV)).cpu()  # NHWC
    base = _oracle_sub('n6').base
    with torch.no_grad():
        img = ofe.resize_bilinear(maps.unsqueeze(1), (512, 512)).repeat(1, 3, 1, 1)
        ref = base.maxpool(base.act1(base.bn1(base.conv1(img)))).permute(0, 2, 3, 1)
    err = ((out - ref).abs().max() / ref.abs().max()).item()
    print(f'stem fp32 rel err {err:.3e}')
    assert err <= 1e-5


def test_stem_bf16_vs_oracle(golden_frontend):
    """bf16 stem (8x8 tap grid, LDS band, register vertical max) vs the fp32 oracle."""
    from oracle import frontend as ofe
    from sad.engine import Backbone, split_merged_state
    _, bases, _ = split_merged_state(merged_sd('n6'))
    bb = Backbone(bases[0], DEV, 'bf16')
    maps = torch.from_numpy(golden_frontend['std_map'])
    out = bb.stem(maps.to(DEV)).float().cpu()
    base = _oracle_sub('n6').base
    with torch.no_grad():
        img = ofe.resize_bilinear(maps.unsqueeze(1), (512, 512)).repeat(1, 3, 1, 1)
        ref = base.maxpool(base.act1(base.bn1(base.conv1(img)))).permute(0, 2, 3, 1)
    err = ((out - ref).abs().max() / ref.abs().max()).item()
    print(f'stem bf16 rel err {err:.3e}')
    assert err <= 2e-2


@pytest.mark.parametrize('dtype,tol', [('fp32', 1e-4), ('bf16', 6e-2)])
def test_backbone_vs_oracle(golden_frontend, golden_models, dtype, tol):
    from sad.engine import Backbone, split_merged_state
    sd = merged_sd('n6')
    _, bases, _ = split_merged_state(sd)
    bb = Backbone(bases[0], DEV, dtype)
    maps = torch.from_numpy(golden_frontend['std_map']).to(DEV)
    feats, l4 = bb.debug(maps)
    ref = torch.from_numpy(golden_models['n6_feats0'])
    err = ((feats.cpu() - ref).abs().max() / ref.abs().max()).item()
    print(f'backbone {dtype} pooled-feature rel err {err:.3e}')
    assert err <= tol


@pytest.mark.parametrize('tag', ['n6', 'n2'])
def test_logits_fp32_match_reference(golden_frontend, golden_models, tag):
    """North-star gate: end to end from int16 PCM, fp32 mode, |dlogit| <= 1e-3."""
    from sad.engine import Engine
    eng = Engine(merged_sd(tag), DEV, dtype='fp32', micro_batch=4)
    assert len(eng.backbones) == (1 if tag == 'n6' else 2)
    pcm = torch.from_numpy(golden_frontend['pcm']).to(DEV)
    logits, merged = eng.forward_pcm(pcm)
    torch.cuda.synchronize()
    d_merged = np.abs(merged.cpu().numpy() - golden_models[f'{tag}_merged']).max()
    d_heads = np.abs(logits.cpu().numpy() - golden_models[f'{tag}_per_head']).max()
    print(f'{tag} fp32 max|dlogit| merged {d_merged:.3e} per-head {d_heads:.3e}')
    assert d_merged <= 1e-3 and d_heads <= 1e-3


def test_logits_bf16_deviation(golden_frontend, golden_models):
    from sad.engine import Engine
    eng = Engine(merged_sd('n6'), DEV, dtype='bf16', micro_batch=4)
    pcm = torch.from_numpy(golden_frontend['pcm']).to(DEV)
    _, merged = eng.forward_pcm(pcm)
    d = np.abs(merged.cpu().numpy() - golden_models['n6_merged']).max()
    print(f'n6 bf16 max|dlogit| {d:.3e}')
    assert d <= 1e-1


def test_decisions_bit_exact(golden_frontend, golden_models):
    from oracle.decision import interpret_multihead_logits
    from sad.engine import Engine
    eng = Engine(merged_sd('n6'), DEV, dtype='fp32', micro_batch=4)
    _, merged = eng.forward_pcm(torch.from_numpy(golden_frontend['pcm']).to(DEV))
    names = [f'Synthetic{chr(65 + i)}' for i in range(6)]
    for row, ref in zip(merged.cpu(), torch.from_numpy(golden_models['n6_merged'])):
        assert interpret_multihead_logits(row, 0.5, names)[0] == interpret_multihead_logits(ref, 0.5, names)[0]


def test_microbatch_invariance():
    """B not a multiple of the micro-batch, ragged tail; results independent of chunking."""
    from sad.engine import Backbone, split_merged_state
    from sad import _lib
    sd = merged_sd('n6')
    _, bases, _ = split_merged_state(sd)
    fe_ = __import__('sad.engine', fromlist=['FrontEnd']).FrontEnd(DEV)
    pcm = torch.empty(37, 128000, dtype=torch.int16, device=DEV)
    _lib.call('sad_synth_pcm', 3, 0, 37, 128000, _lib.ptr(pcm), _lib.stream_handle(torch.device(DEV)))
    maps = fe_(pcm)
    a = Backbone(bases[0], DEV, 'bf16', micro_batch=16)(maps)
    b = Backbone(bases[0], DEV, 'bf16', micro_batch=37)(maps)
    assert torch.equal(a, b)


@pytest.mark.parametrize('dtype,tol', [('fp32', 1e-5), ('bf16', 4e-3)])
def test_fused_avgpool_matches_separate_pool(dtype, tol):
    """The last layer4 conv pools its relu(acc + bias) tiles itself (fused global
    average pool, fp32 sums); the debug path stores the layer4 map (bf16 in the
    throughput mode) and runs the separate avgpool kernel.  fp32: summation
    order only; bf16: the stored map's rounding (2^-9 relative per element)."""
    from sad.engine import Backbone, split_merged_state
    from sad import _lib
    _, bases, _ = split_merged_state(merged_sd('n6'))
    fe_ = __import__('sad.engine', fromlist=['FrontEnd']).FrontEnd(DEV)
    pcm = torch.empty(9, 128000, dtype=torch.int16, device=DEV)
    _lib.call('sad_synth_pcm', 7, 0, 9, 128000, _lib.ptr(pcm), _lib.stream_handle(torch.device(DEV)))
    maps = fe_(pcm)
    bb = Backbone(bases[0], DEV, dtype, micro_batch=9)
    fused = bb(maps)
    sep, l4 = bb.debug(maps)
    torch.cuda.synchronize()
    ref = l4.float().mean(dim=(1, 2))
    assert torch.allclose(sep, ref, rtol=1e-5, atol=1e-5)
    err = ((fused - sep).abs().max() / sep.abs().max()).item()
    assert err <= tol, err
