"""GPU parity on the 16-segment reference fixture (tests/golden/
make_golden_models16.py: logits by the reference's own load_merged_model +
ModularMultiHeadClassifier) including a 6-head model on 6 DISTINCT backbones,
and on 32 segments of the configs[1] 1,024-segment batch against the CPU
oracle (every micro-batch boundary of the fp32 and split-bf16 plans, plus
clipped / quiet / near-silent edge segments).

Tolerance: |dlogit| <= 1e-3 (north star) for the fp32 and bf16x3 modes; the
implied decisions must be identical.
"""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN, merged_sd

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'
sys.path.insert(0, GOLDEN)


def _sd(tag):
    from sad import weights as sw
    n, distinct, seed = {'n6': (6, False, 0), 'n2': (2, True, 1), 'n6d': (6, True, 2)}[tag]
    return sw.merged_state_dict(seed, n, distinct, bn_stats=sw.load_bn_stats(os.path.join(GOLDEN, f'bn_stats_{tag}.npz')))


@pytest.fixture(scope='module')
def seg16():
    from make_golden_models16 import segments16
    pcm = segments16()
    fx = dict(np.load(os.path.join(GOLDEN, 'golden_models16.npz')))
    assert int(pcm.astype(np.int64).sum()) == int(fx['pcm_sum'][0])
    assert int(np.abs(pcm.astype(np.int64)).sum()) == int(fx['pcm_abs_sum'][0])
    return pcm, fx


@pytest.mark.parametrize('dtype', ['fp32', 'bf16x3'])
@pytest.mark.parametrize('tag', ['n6', 'n2', 'n6d'])
def test_logits16_match_reference(seg16, tag, dtype):
    from oracle.decision import interpret_multihead_logits
    from sad.engine import Engine
    pcm, fx = seg16
    eng = Engine(_sd(tag), DEV, dtype=dtype, micro_batch=5)  # 16 = 5 + 5 + 5 + 1
    assert len(eng.backbones) == {'n6': 1, 'n2': 2, 'n6d': 6}[tag]
    logits, merged = eng.forward_pcm(torch.from_numpy(pcm).to(DEV))
    torch.cuda.synchronize()
    dm = np.abs(merged.cpu().numpy() - fx[f'{tag}_merged']).max()
    dh = np.abs(logits.cpu().numpy() - fx[f'{tag}_per_head']).max()
    print(f'{tag} {dtype}: max|dlogit| merged {dm:.3e} per-head {dh:.3e}')
    assert dm <= 1e-3 and dh <= 1e-3
    n = eng.n_heads
    names = [f'S{i}' for i in range(n)]
    for row, ref in zip(merged.cpu(), torch.from_numpy(fx[f'{tag}_merged'])):
        assert interpret_multihead_logits(row, 0.5, names)[0] == interpret_multihead_logits(ref, 0.5, names)[0]


def _batch1024():
    """configs[1]: 1,024 device-synthesised segments (seed 11) with edge cases
    written over a few of them; returns (device pcm, indices to check)."""
    from sad import _lib
    n = 1024
    pcm = torch.empty(n, 128000, dtype=torch.int16, device=DEV)
    _lib.call('sad_synth_pcm', 11, 0, n, 128000, _lib.ptr(pcm), _lib.stream_handle(torch.device(DEV)))
    host = pcm[[40, 300, 600, 900]].cpu().to(torch.int64)
    edits = {40: (host[0] * 16).clamp(-32768, 32767), 300: host[1] // 100, 600: host[2] // 1000,
             900: torch.where(host[3] >= 0, 32767, -32768)}
    for i, v in edits.items():
        pcm[i] = v.to(torch.int16).to(DEV)
    bounds = [0, 1, 127, 128, 129, 255, 256, 383, 384, 511, 512, 513, 639, 640, 767, 768, 895, 896, 1022, 1023]
    idx = sorted(set(bounds + list(edits) + [17, 222, 333, 444, 555, 666, 777, 888]))
    assert len(idx) >= 32
    return pcm, idx


@pytest.mark.parametrize('dtype,mb', [('fp32', 128), ('bf16x3', 256)])
def test_logits_batch1024_vs_oracle(dtype, mb):
    from oracle import frontend as ofe
    from oracle import resnet as ores
    from sad.engine import Engine
    sd = merged_sd('n6')
    pcm, idx = _batch1024()
    _, merged = Engine(sd, DEV, dtype=dtype, micro_batch=mb).forward_pcm(pcm)
    torch.cuda.synchronize()
    model = ores.load_merged_state(sd)
    sub = pcm[idx].cpu()
    with torch.no_grad():
        imgs = torch.cat([ofe.waveform_to_spectrogram(sub[i].to(torch.float32) / 32768.0, 32000,
                                                      ofe.SpectrogramConfig()) for i in range(len(idx))])
        ref = model(imgs)
    d = (merged[idx].cpu() - ref).abs().max().item()
    print(f'{dtype}: 1024-segment batch, {len(idx)} segments vs oracle: max|dlogit| {d:.3e}')
    assert d <= 1e-3
    assert torch.isfinite(merged).all()
