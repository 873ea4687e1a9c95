"""Is the compute stream's first libsad launch after torch's wait_event
ordered behind the side stream's front end?  bench.Mode's pipelined sequence,
20 reps each: (a) as is; (b) a tiny torch kernel on the compute stream between
the wait and the backbone; (c) hipStreamWaitEvent issued again by libsad's
caller... via cur.wait_stream(side) as well."""
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
tick = torch.zeros(1, device=dev)


def run(variant):
    ovl = bench.Mode(sd, dev, 'bf16', 64, B, 1, overlap=True)
    bb = ovl.eng.backbones[0]
    if variant in ('sleep_before_record', 'record_twice'):
        orig_fa = ovl._frontend_ahead

        def fa(pcm, slot, ev=None):
            ovl.side.wait_event(ovl.bb_done[slot])
            with torch.cuda.stream(ovl.side):
                ovl.maps[slot] = ovl.eng.frontend(pcm, out=ovl.maps[slot])
            if variant == 'sleep_before_record':
                import time
                time.sleep(0.002)
            ovl.fe_done[slot].record(ovl.side)
            if variant == 'record_twice':
                ovl.fe_done[slot].record(ovl.side)
        ovl._frontend_ahead = fa

    class BB:
        def __call__(self, m, out=None):
            if variant == 'tick':
                tick.add_(1)
            elif variant == 'wait_stream':
                torch.cuda.current_stream().wait_stream(ovl.side)
            return bb(m, out=out)
    ovl.eng.backbones[0] = BB()
    got = []
    torch.cuda.synchronize()
    for i, k in enumerate(order):
        nxt = pcms[order[i + 1]] if i + 1 < len(order) else pcms[k]
        ovl.step(pcms[k], next_pcm=nxt)
        got.append(ovl.merged.clone())
    torch.cuda.synchronize()
    return [i for i, k in enumerate(order) if not torch.equal(got[i], ref[k])]


for v in ('as is', 'sleep_before_record', 'record_twice', 'wait_stream'):
    res = [run(v) for _ in range(20)]
    print(f'{v:12s}: {sum(1 for r in res if r)} of 20 reps fail {res}', flush=True)
