"""GPU: bench.py's overlapped front end (--overlap-frontend 1: each step's mel
front end runs on a side stream during the previous step's backbone, two map
buffers).  Every step must still see its own batch's maps: driven with
alternating batches (step i processes batch i and starts batch i+1's front
end), the merged logits of every pipelined step equal the sequential step's
for that batch, bit for bit -- a stale or half-written map buffer would show.
The pipelined steps run back to back with no host synchronisation between
them (each step's logits are copied out on the compute stream), so a missing
wait on fe_done / bb_done or a map-buffer reuse race is free to show up."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_overlapped_frontend_matches_sequential():
    sys.path.insert(0, ROOT)
    import bench
    from sad import _lib
    from sad import weights as sw
    dev = torch.device('cuda:0')
    sd = sw.merged_state_dict(0, bench.HEADS, False,
                              bn_stats=sw.load_bn_stats(os.path.join(ROOT, 'tests', 'golden', 'bn_stats_n6.npz')))
    B = 96
    pcms = []
    for seed in (3, 4):
        p = torch.empty(B, bench.SEG, dtype=torch.int16, device=dev)
        _lib.call('sad_synth_pcm', seed, 0, B, bench.SEG, _lib.ptr(p), _lib.stream_handle(dev))
        pcms.append(p)
    seq = bench.Mode(sd, dev, 'bf16', 64, B, 1)
    ref = []
    for p in pcms:
        seq.step(p)
        torch.cuda.synchronize()
        ref.append(seq.merged.clone())
    assert not torch.equal(ref[0], ref[1])
    order = [0, 1, 1, 0, 1, 0, 0]
    # 8 repetitions of the sequence: a cross-stream ordering hole shows in a
    # fraction of them (before the fix in bench.Mode.step: 25-55 % of the
    # repetitions had a step reading a half-written map)
    for rep in range(8):
        ovl = bench.Mode(sd, dev, 'bf16', 64, B, 1, overlap=True)
        got = []
        torch.cuda.synchronize()
        for i, k in enumerate(order):
            nxt = pcms[order[i + 1]] if i + 1 < len(order) else pcms[k]
            ovl.step(pcms[k], next_pcm=nxt)
            got.append(ovl.merged.clone())  # on the compute stream, after this step's heads
        torch.cuda.synchronize()
        for i, k in enumerate(order):
            assert torch.equal(got[i], ref[k]), f'repetition {rep}, step {i}'
