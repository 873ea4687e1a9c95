"""tools/overlap_repeat.py's pipelined sequence in two forms, 20 reps each:
(a) bench.Mode as is (two events per kind, re-recorded every other step);
(b) fresh events for every record.  Counts the steps whose logits differ from
the sequential step's."""
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


class FreshEvents(list):
    """fe_done / bb_done with a new event at every record (record() replaced)."""


def run(mode_fresh):
    ovl = bench.Mode(sd, dev, 'bf16', 64, B, 1, overlap=True)
    if mode_fresh:
        orig = ovl._frontend_ahead

        def fa(pcm, slot, ev=None):
            ovl.fe_done[slot] = torch.cuda.Event()
            return orig(pcm, slot, ev)
        ovl._frontend_ahead = fa
        orig_bb = ovl.eng.backbones[0]

        class BB:
            def __call__(self, m, out=None):
                r = orig_bb(m, out=out)
                ovl.bb_done[ovl.i & 1] = torch.cuda.Event()
                return r
        ovl.eng.backbones[0] = BB()
    got = []
    torch.cuda.synchronize()
    for i, k in enumerate(order):
        nxt = pcms[order[i + 1]] if i + 1 < len(order) else pcms[k]
        ovl.step(pcms[k], next_pcm=nxt)
        got.append(ovl.merged.clone())
    torch.cuda.synchronize()
    return [i for i, k in enumerate(order) if not torch.equal(got[i], ref[k])]


for fresh in (False, True):
    res = [run(fresh) for _ in range(20)]
    print('fresh events' if fresh else 'bench.Mode as is', 'failing steps:', res,
          'reps with a failure:', sum(1 for r in res if r), flush=True)
