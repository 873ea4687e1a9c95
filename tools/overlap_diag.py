"""Where does the pipelined (side-stream front end) bench step diverge from
the sequential one?  Per step: the maps the backbone reads, the pooled
features and the merged logits, all copied out on the compute stream with no
host synchronisation between steps, against the sequential step of that batch;
the sequential reference is run twice (determinism)."""
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


def seq_run():
    seq = bench.Mode(sd, dev, 'bf16', 64, B, 1)
    out = []
    for p in pcms:
        m = seq.eng.frontend(p)
        seq.eng.backbones[0](m, out=seq.feats)
        seq.eng.heads([seq.feats], seq.logits, seq.merged)
        torch.cuda.synchronize()
        out.append((m.clone(), seq.feats.clone(), seq.merged.clone()))
    return out


r1, r2 = seq_run(), seq_run()
print('sequential deterministic:', [all(torch.equal(a, b) for a, b in zip(x, y)) for x, y in zip(r1, r2)])
order = [0, 1, 1, 0, 1, 0, 0, 1, 0, 0, 1, 1]
for rep in range(int(os.environ.get('REPS', '20'))):
    ovl = bench.Mode(sd, dev, 'bf16', 64, B, 1, overlap=True)
    got = []
    torch.cuda.synchronize()
    for i, k in enumerate(order):
        nxt = pcms[order[i + 1]] if i + 1 < len(order) else pcms[k]
        slot = ovl.i & 1
        if ovl.i == 0:
            ovl._frontend_ahead(pcms[k], slot)
        cur = torch.cuda.current_stream()
        cur.wait_event(ovl.fe_done[slot])
        mcopy = ovl.maps[slot].clone()
        ovl.eng.backbones[0](ovl.maps[slot], out=ovl.feats)
        ovl.bb_done[slot].record(cur)
        fcopy = ovl.feats.clone()
        ovl.eng.heads([ovl.feats], ovl.logits, ovl.merged)
        got.append((mcopy, fcopy, ovl.merged.clone()))
        ovl._frontend_ahead(nxt, slot ^ 1)
        ovl.i += 1
    torch.cuda.synchronize()
    res = []
    for i, k in enumerate(order):
        eq = [torch.equal(a, b) for a, b in zip(got[i], r1[k])]
        d = [(a.float() - b.float()).abs().max().item() for a, b in zip(got[i], r1[k])]
        if all(eq):
            res.append('ok')
            continue
        segm = ((got[i][0] - r1[k][0]).abs().amax(dim=(1, 2)) > 0).nonzero().flatten().tolist()
        segf = ((got[i][1] - r1[k][1]).abs().amax(dim=1) > 0).nonzero().flatten().tolist()
        other = r1[1 - k][0]
        stale = []
        for sgi in segm[:3]:
            dm = (got[i][0][sgi] != r1[k][0][sgi])
            st = (got[i][0][sgi] == other[sgi]) & dm
            rows = sorted(set(dm.nonzero()[:, 0].tolist()))
            stale.append((sgi, int(dm.sum()), int(st.sum()), rows[:6]))
        res.append(f'step{i}: maps {eq[0]} feats {eq[1]} merged {eq[2]} d={d} map-segs {segm[:8]} feat-segs {segf[:8]} '
                   f'(seg, differing, equal-to-other-batch, rows) {stale}')
    print(f'rep {rep}:', [r for r in res if r != 'ok'] or 'all steps equal')
