"""The pipelined bench step (bench.Mode with overlap) 20 times each with the
compute on (a) torch's default stream, (b) a created stream; then (c) on the
default stream with the front end's map buffers allocated by the compute
stream.  Counts reps with a step whose logits differ from the sequential step."""
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


def run(prealloc):
    ovl = bench.Mode(sd, dev, 'bf16', 64, B, 1, overlap=True)
    if prealloc:
        ovl.maps = [torch.empty(B, 128, 251, device=dev) for _ in range(2)]
    got = []
    torch.cuda.synchronize()
    for i, k in enumerate(order):
        nxt = pcms[order[i + 1]] if i + 1 < len(order) else pcms[k]
        ovl.step(pcms[k], next_pcm=nxt)
        got.append(ovl.merged.clone())
    torch.cuda.synchronize()
    return [i for i, k in enumerate(order) if not torch.equal(got[i], ref[k])]


res = [run(False) for _ in range(20)]
print('(a) default stream:', sum(1 for r in res if r), 'of 20 reps fail', res, flush=True)
s_main = torch.cuda.Stream(dev)
with torch.cuda.stream(s_main):
    res = [run(False) for _ in range(20)]
torch.cuda.synchronize()
print('(b) created stream:', sum(1 for r in res if r), 'of 20 reps fail', res, flush=True)
res = [run(True) for _ in range(20)]
print('(c) maps allocated on the compute stream:', sum(1 for r in res if r), 'of 20 reps fail', res, flush=True)
