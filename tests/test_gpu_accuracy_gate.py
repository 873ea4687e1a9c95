"""GPU accuracy gate at the bench's configs[2] workload:
B = 2,048 synthetic segments (sad_synth_pcm, seed 0, the bench's rank-0 batch),
6-head ensemble (the golden n6 model), bf16 at micro-batch 1,024 and at the
bench's 2,048 and the split-bf16 parity mode at 256 and at the bench's 512 (its
layer1 output is 512 x 128^2 x 128 x 2 B = 2^31 B, so layer2.0's convs run as
split-bf16 image-range launches), each against the fp32 device path (f32
MFMA, itself within 3.1e-5 of the reference fixtures, test_gpu_parity.py).

Gates:
  * bf16x3 (parity mode): max|dlogit| <= 1e-3 (north star) and every decision
    identical -- the numbers bench.py reports as parity_mode.accuracy;
  * bf16 (the headline): max|dlogit| <= 0.15 and >= 95 % identical decisions --
    bench.py's accuracy line (measured 0.087 and 97.3 % in round 2).  bf16 does
    not meet the north star's 1e-3: tools/error_budget.py shows that rounding
    ANY single conv's weights or activations to bf16 already moves the logits by
    6e-3 .. 3.7e-2, so no mixed bf16 / split-bf16 plan meets it.

Decisions: interpret_multihead_logits (inference_runner.py:194-214) on the
merged logits, threshold 0.5, as bench.py's decisions().
"""
import os

import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'
B = 2048


@pytest.fixture(scope='module')
def batch():
    from sad import _lib
    from sad import weights as sw
    from sad.engine import Engine
    sd = sw.merged_state_dict(0, 6, False, bn_stats=sw.load_bn_stats(os.path.join(GOLDEN, 'bn_stats_n6.npz')))
    pcm = torch.empty(B, 128000, dtype=torch.int16, device=DEV)
    _lib.call('sad_synth_pcm', 0, 0, B, 128000, _lib.ptr(pcm), _lib.stream_handle(torch.device(DEV)))
    _, m32 = Engine(sd, DEV, dtype='fp32', micro_batch=128).forward_pcm(pcm)
    torch.cuda.synchronize()
    return sd, pcm, m32.cpu()


def _decisions(merged):
    import inference_runner as ir
    names = [f'Synthetic{chr(65 + i)}' for i in range(6)]
    return [ir.interpret_multihead_logits(row, 0.5, names)[0] for row in merged]


@pytest.mark.parametrize('dtype,mb,dmax,agree_min', [('bf16x3', 256, 1e-3, 1.0), ('bf16x3', 512, 1e-3, 1.0),
                                                     ('bf16', 1024, 0.15, 0.95), ('bf16', 2048, 0.15, 0.95)])
def test_configs2_accuracy_vs_fp32_device(batch, dtype, mb, dmax, agree_min):
    from sad.engine import Engine
    sd, pcm, m32 = batch
    _, m = Engine(sd, DEV, dtype=dtype, micro_batch=mb).forward_pcm(pcm)
    torch.cuda.synchronize()
    m = m.cpu()
    assert torch.isfinite(m).all()
    d = (m - m32).abs().max().item()
    l32, lm = _decisions(m32), _decisions(m)
    agree = sum(a == b for a, b in zip(lm, l32)) / B
    print(f'{dtype} mb {mb}: max|dlogit| vs fp32 device {d:.3e}, decisions identical {agree:.4f}')
    assert d <= dmax, d
    assert agree >= agree_min, agree
