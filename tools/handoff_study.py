"""Round-5 study of a cross-stream hand-off: the front end of
step s+1 on a side stream during step s's backbone, two map slots, as
bench.Mode ran it in round 4 (+0.9 %).  Each form drives the same 7-step
sequence of two batches 40 times and counts the repetitions in which some
step's merged logits differ from the sequential step's (bit-exact compare).

  event   compute stream waits on the front end's event (round 4's code)
  host    + the host waits on that event before enqueueing the backbone
  acquire + an agent-scope acquire (buffer_inv sc1) in 4096 workgroups on
          the compute stream before the backbone (tools/fence_diag.hip)
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


class Pipelined(bench.Mode):
    def __init__(self, form):
        super().__init__(sd, dev, 'bf16', MB, B, 1)
        self.form = form
        self.side = torch.cuda.Stream(dev)
        self.maps = [None, None]
        self.fe_done = [torch.cuda.Event(), torch.cuda.Event()]
        self.bb_done = [torch.cuda.Event(), torch.cuda.Event()]
        self.i = 0

    def ahead(self, pcm, slot):
        self.side.wait_event(self.bb_done[slot])
        with torch.cuda.stream(self.side):
            self.maps[slot] = self.eng.frontend(pcm, out=self.maps[slot])
        self.fe_done[slot].record(self.side)

    def pstep(self, pcm, nxt):
        slot = self.i & 1
        if self.i == 0:
            self.ahead(pcm, slot)
        cur = torch.cuda.current_stream()
        cur.wait_event(self.fe_done[slot])
        if self.form == 'host':
            self.fe_done[slot].synchronize()
        if self.form == 'acquire':
            assert fl.fence_launch(0, 4096, None, cur.cuda_stream) == 0
        self.eng.backbones[0](self.maps[slot], out=self.feats)
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
    ref = []
    for p in pcms:
        seq.step(p)
        torch.cuda.synchronize()
        ref.append(seq.merged.clone())

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
        return [i for i, k in enumerate(ORDER) if not torch.equal(got[i], ref[k])]

    for form in sys.argv[1:] or ['event', 'host', 'acquire', 'serial', 'nohand']:
        res = [run(form) for _ in range(40)]
        print(f'{form:8s}: {sum(1 for r in res if r):2d} of 40 repetitions differ; failing steps '
              f'{sorted({s for r in res for s in r})}', flush=True)


if __name__ == '__main__':
    main()
