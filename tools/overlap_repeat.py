"""Repeat tests/test_gpu_bench_overlap.py's pipelined sequence (bench.Mode.step
with overlap, no host syncs between steps) N times in one process and count
the steps whose logits differ from the sequential step's."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'synthetic-audio-detection_amd')]
import bench  # noqa: E402
from sad import _lib  # noqa: E402
from sad import weights as sw  # noqa: E402

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
order = [0, 1, 1, 0, 1, 0, 0]
fails = []
for rep in range(int(os.environ.get('REPS', '10'))):
    ovl = bench.Mode(sd, dev, 'bf16', 64, B, 1, overlap=True)
    got = []
    torch.cuda.synchronize()
    for i, k in enumerate(order):
        nxt = pcms[order[i + 1]] if i + 1 < len(order) else pcms[k]
        ovl.step(pcms[k], next_pcm=nxt)
        got.append(ovl.merged.clone())
    torch.cuda.synchronize()
    bad = [(i, (got[i] - ref[k]).abs().max().item()) for i, k in enumerate(order) if not torch.equal(got[i], ref[k])]
    fails.append(bad)
print(os.environ.get('SAD_S2_PATCH', 'default'), 'failing steps per rep:', fails, flush=True)
