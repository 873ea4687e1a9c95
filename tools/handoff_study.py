"""Round-5 study of a cross-stream hand-off: the front end of
step s+1 on a side stream during step s's backbone, two map slots, as
bench.Mode ran it in round 4 (+0.9 %).  Each form drives the same 7-step
sequence of two batches 40 times and counts the repetitions in which some
step's merged logits differ from the sequential step's (bit-exact compare).

  event   compute stream waits on the front end's event (round 4's code)
  host    + the host waits on that event before enqueueing the backbone
  acquire + an agent-scope acquire (buffer_inv sc1) in 4096 workgroups on
          the compute stream before the backbone (tools/fence_diag.hip)
  delay   the acquire form's 4096-workgroup grid with no fence (timing only)
  spin    a 4096-workgroup grid that sleeps ~110 us per wave, no fence
  relside an agent-scope release (buffer_wbl2) grid on the SIDE stream after
          the front end, before its event: producer-side write-back
  devsync torch.cuda.synchronize() (every stream) before the backbone
  serial  the next front end starts only after this step's heads finished:
          hand-off, nothing concurrent
  nohand  sequential steps plus a concurrent front end into a scratch buffer
          nobody reads: concurrency, no hand-off

Build the fence kernel first (CPU side):
  hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/fence_diag.hip -o tools/_fence_diag.so"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'synthetic-audio-detection_amd')]
import bench  # noqa: E402
from sad import _lib  # noqa: E402
from sad import weights as sw  # noqa: E402

dev = torch.device('cuda:0')
fl = ctypes.CDLL(os.path.join(ROOT, 'tools', '_fence_diag.so'))
fl.fence_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
sd = sw.merged_state_dict(0, bench.HEADS, False,
                          bn_stats=sw.load_bn_stats(os.path.join(ROOT, 'tests', 'golden', 'bn_stats_n6.npz')))
B, MB = 96, 64
ORDER = [0, 1, 1, 0, 1, 0, 0]
REPS = int(os.environ.get('HANDOFF_REPS', '40'))
FENCE_KIND = {'acquire': 0, 'delay': 3, 'spin': 4}
# HANDOFF_LOCATE=1: per step, compare the map the backbone read (cloned after it
# ran) and its features with the sequential ones, and describe any difference
LOCATE = os.environ.get('HANDOFF_LOCATE', '0') == '1'


class Pipelined(bench.Mode):
    def __init__(self, form):
        super().__init__(sd, dev, 'bf16', MB, B, 1)
        self.form = form
        self.side = torch.cuda.Stream(dev)
        self.maps = [None, None]
        self.fe_done = [torch.cuda.Event(), torch.cuda.Event()]
        self.bb_done = [torch.cuda.Event(), torch.cuda.Event()]
        self.i = 0
        self.seen = []

    def ahead(self, pcm, slot):
        self.side.wait_event(self.bb_done[slot])
        with torch.cuda.stream(self.side):
            self.maps[slot] = self.eng.frontend(pcm, out=self.maps[slot])
        if self.form == 'relside':
            assert fl.fence_launch(1, 4096, None, self.side.cuda_stream) == 0
        self.fe_done[slot].record(self.side)

    def pstep(self, pcm, nxt):
        slot = self.i & 1
        if self.i == 0:
            self.ahead(pcm, slot)
        cur = torch.cuda.current_stream()
        cur.wait_event(self.fe_done[slot])
        if self.form == 'host':
            self.fe_done[slot].synchronize()
        if self.form == 'devsync':
            torch.cuda.synchronize()
        if self.form in FENCE_KIND:
            assert fl.fence_launch(FENCE_KIND[self.form], 4096, None, cur.cuda_stream) == 0
        self.eng.backbones[0](self.maps[slot], out=self.feats)
        if LOCATE:  # what the backbone read and wrote, captured before the slot may be reused
            self.seen.append((self.maps[slot].clone(), self.feats.clone()))
        self.bb_done[slot].record(cur)
        self.eng.heads([self.feats], self.logits, self.merged)
        if self.form == 'serial':
            cur.synchronize()
        self.ahead(nxt, slot ^ 1)
        self.i += 1


def main():
    pcms = []
    for seed in (3, 4):
        p = torch.empty(B, bench.SEG, dtype=torch.int16, device=dev)
        _lib.call('sad_synth_pcm', seed, 0, B, bench.SEG, _lib.ptr(p), _lib.stream_handle(dev))
        pcms.append(p)
    seq = bench.Mode(sd, dev, 'bf16', MB, B, 1)
    ref, ref_map, ref_feat, ref_db = [], [], [], []
    for p in pcms:
        seq.step(p)
        torch.cuda.synchronize()
        ref.append(seq.merged.clone())
        ref_feat.append(seq.feats.clone())
        ref_map.append(seq.eng.frontend(p).clone())  # the in-place form the pipeline runs
        ref_db.append(seq.eng.frontend(p, want_db=True)[1].clone())
    torch.cuda.synchronize()

    def describe(i, k, mp, ft, mg):
        """One failing step: which tensors differ, where, and what the wrong map values are."""
        out = [f'  step {i} (batch {k}, slot {i & 1}):']
        dm = (mp != ref_map[k])
        if dm.any():
            segs = dm.flatten(1).any(1).nonzero().flatten().tolist()
            idx = dm.nonzero()
            out.append(f'    map differs: {int(dm.sum())} elements in segments {segs[:8]}, rows '
                       f'{idx[:, 1].min().item()}..{idx[:, 1].max().item()}, cols {idx[:, 2].min().item()}..'
                       f'{idx[:, 2].max().item()}; max |d| {(mp - ref_map[k]).abs().max().item():.3g}')
            flat = dm.flatten().nonzero().flatten()
            lines = sorted({int(x) // 32 for x in flat.tolist()})
            out.append(f'    differing 128-B lines: {len(lines)} (first {lines[:6]})')
            wrong = mp.flatten()[flat]
            out.append(f'    wrong values equal: other batch map {bool((wrong == ref_map[1 - k].flatten()[flat]).all())}, '
                       f'this batch dB {bool((wrong == ref_db[k].flatten()[flat]).all())}, '
                       f'other batch dB {bool((wrong == ref_db[1 - k].flatten()[flat]).all())}')
        else:
            out.append('    map (cloned after the backbone) equals the sequential map')
        df = (ft != ref_feat[k])
        if df.any():
            out.append(f'    feats differ in segments {df.any(1).nonzero().flatten().tolist()[:8]}, '
                       f'max |d| {(ft - ref_feat[k]).abs().max().item():.3g}')
        else:
            out.append('    feats equal')
        out.append(f'    merged max |d| {(mg - ref[k]).abs().max().item():.3g}')
        return '\n'.join(out)

    def run(form):
        got = []
        torch.cuda.synchronize()
        if form == 'nohand':
            side = torch.cuda.Stream(dev)
            scratch = torch.empty(B, 128, 251, device=dev)
            for i, k in enumerate(ORDER):
                seq.step(pcms[k])
                with torch.cuda.stream(side):
                    seq.eng.frontend(pcms[ORDER[min(i + 1, len(ORDER) - 1)]], out=scratch)
                got.append(seq.merged.clone())
        else:
            m = Pipelined(form)
            for i, k in enumerate(ORDER):
                m.pstep(pcms[k], pcms[ORDER[i + 1]] if i + 1 < len(ORDER) else pcms[k])
                got.append(m.merged.clone())
        torch.cuda.synchronize()
        bad = [i for i, k in enumerate(ORDER) if not torch.equal(got[i], ref[k])]
        if LOCATE and form != 'nohand':
            for i in bad:
                print(describe(i, ORDER[i], m.seen[i][0], m.seen[i][1], got[i]), flush=True)
        return bad

    cur = torch.cuda.current_stream()
    for kind in (0, 3, 4, 1):
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(3):
            t0.record(cur)
            assert fl.fence_launch(kind, 4096, None, cur.cuda_stream) == 0
            t1.record(cur)
        torch.cuda.synchronize()
        print(f'fence kind {kind}: {t0.elapsed_time(t1) * 1e3:.1f} us per 4096-workgroup launch', flush=True)
    for form in sys.argv[1:] or ['event', 'host', 'acquire', 'delay', 'spin', 'relside', 'devsync', 'serial',
                                 'nohand']:
        res = [run(form) for _ in range(REPS)]
        print(f'{form:8s}: {sum(1 for r in res if r):2d} of {REPS} repetitions differ; failing steps '
              f'{sorted({s for r in res for s in r})}', flush=True)


if __name__ == '__main__':
    main()
