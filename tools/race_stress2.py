"""The front end's determinism while the backbone (and its kernels one by one)
run concurrently on another stream: the FE output map is compared bit for bit
with a quiet-device reference.  (tools/race_stress.py checks the converse.)"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'synthetic-audio-detection_amd')]
from sad import weights as sw  # noqa: E402
from sad.engine import Backbone, FrontEnd, split_merged_state  # noqa: E402

DEV = torch.device('cuda:0')
REPS = int(os.environ.get('REPS', '20'))
g = torch.Generator(device=DEV).manual_seed(2)
side = torch.cuda.Stream(DEV)
fe = FrontEnd(DEV)
pcm = torch.randint(-20000, 20000, (96, 128000), dtype=torch.int16, device=DEV, generator=g)
sd = sw.merged_state_dict(0, 6, False, bn_stats=sw.load_bn_stats(os.path.join(ROOT, 'tests', 'golden', 'bn_stats_n6.npz')))
_, bases, _ = split_merged_state(sd)
bb = Backbone(bases[0], DEV, 'bf16', micro_batch=64)
bmaps = fe(torch.randint(-20000, 20000, (96, 128000), dtype=torch.int16, device=DEV, generator=g))
ref_m, ref_db = fe(pcm, want_db=True)
ref_m, ref_db = ref_m.clone(), ref_db.clone()
torch.cuda.synchronize()
bad = 0
for r in range(REPS):
    with torch.cuda.stream(side):
        for _ in range(2):
            bb(bmaps)
    # start the front end a little into the backbone (as the bench's side stream does)
    torch.cuda._sleep(20000 * (r % 5))
    m, db = fe(pcm, want_db=True)
    torch.cuda.synchronize()
    okm, okd = torch.equal(m, ref_m), torch.equal(db, ref_db)
    if not (okm and okd):
        bad += 1
        d = (m - ref_m).abs()
        e = (db - ref_db).abs()
        seg = (e.amax(dim=(1, 2)) > 0).nonzero().flatten().tolist()
        print(f'rep {r}: map equal {okm}, dB equal {okd}; dB max diff {e.max().item():.3g} in segments {seg[:10]}; '
              f'map max diff {d.max().item():.3g}', flush=True)
        if seg:
            s0 = seg[0]
            loc = (e[s0] > 0).nonzero()
            print(f'   segment {s0}: {len(loc)} dB values differ, mel rows {sorted(set(loc[:, 0].tolist()))[:20]}, '
                  f'frames {sorted(set(loc[:, 1].tolist()))[:40]}', flush=True)
print(f'front end under a concurrent backbone: {REPS - bad}/{REPS} bit-identical', flush=True)
