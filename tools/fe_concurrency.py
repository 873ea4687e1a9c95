"""Round-6 follow-up to tools/handoff_study.py: the pipelined
hand-off's wrong logits come from wrong MAPS -- two adjacent mel rows of one
frame, or one segment's standardisation -- produced by a front end that ran
while the backbone's first kernels ran on another stream.  This drives the
front end (96 segments, in place as the bench runs it, and with a separate dB
buffer) on the main stream while one candidate kernel runs on a side stream,
REPS times each, and counts maps that differ bit for bit from a quiet run.

  none      nothing concurrent
  stem      sad_backbone_stem_run (96 segments), the backbone's first kernel
  backbone  the whole backbone
  lds       a kernel that only reads / writes its own 81,696 B of LDS (the
            stem's footprint), 256 threads: co-residency without the stem's code
  copy      large device-to-device copies (memory traffic, no LDS)
  bperm / mfma / dpp / mix   probe_kernel: ONE feature of the stem (ds_bpermute,
            MFMA chains, DPP + packed-int16 max, or all three) at the stem's LDS
            footprint

Build the probe kernels first (CPU side):
  hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/fence_diag.hip -o tools/_fence_diag.so"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'synthetic-audio-detection_amd')]
from sad import _lib  # noqa: E402
from sad import weights as sw  # noqa: E402
from sad.engine import Backbone, FrontEnd, split_merged_state  # noqa: E402

DEV = torch.device('cuda:0')
REPS = int(os.environ.get('REPS', '40'))
B = 96
DUMP = os.environ.get('FE_DUMP', '')
fl = ctypes.CDLL(os.path.join(ROOT, 'tools', '_fence_diag.so'))
fl.lds_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
fl.probe_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
PROBES = {'bperm': 0, 'mfma': 1, 'dpp': 2, 'mix': 3}


def main():
    g = torch.Generator(device=DEV).manual_seed(5)
    side = torch.cuda.Stream(DEV)
    fe = FrontEnd(DEV)
    pcm = torch.empty(B, 128000, dtype=torch.int16, device=DEV)
    _lib.call('sad_synth_pcm', 3, 0, B, 128000, _lib.ptr(pcm), _lib.stream_handle(DEV))
    sd = sw.merged_state_dict(0, 6, False,
                              bn_stats=sw.load_bn_stats(os.path.join(ROOT, 'tests', 'golden', 'bn_stats_n6.npz')))
    _, bases, _ = split_merged_state(sd)
    bb = Backbone(bases[0], DEV, 'bf16', micro_batch=64)
    bmaps = fe(torch.randint(-20000, 20000, (B, 128000), dtype=torch.int16, device=DEV, generator=g))
    big_a = torch.empty(512 << 20, dtype=torch.uint8, device=DEV)
    big_b = torch.empty_like(big_a)
    ref = fe(pcm).clone()
    ref_m2, ref_db = [t.clone() for t in fe(pcm, want_db=True)]
    out = torch.empty_like(ref)
    db = torch.empty_like(ref)
    torch.cuda.synchronize()

    def noise(kind):
        with torch.cuda.stream(side):
            if kind == 'stem':
                for _ in range(2):
                    bb.stem(bmaps)
            elif kind == 'backbone':
                bb(bmaps)
            elif kind == 'lds':
                assert fl.lds_launch(4096, 81696, 8, side.cuda_stream) == 0
            elif kind in PROBES:  # one stem feature, the stem's LDS footprint (tools/fence_diag.hip probe_kernel)
                assert fl.probe_launch(4096, 81696, PROBES[kind], 4000, side.cuda_stream) == 0
            elif kind == 'copy':
                for _ in range(2):
                    big_b.copy_(big_a)

    for kind in (sys.argv[1:] or ['none', 'stem', 'lds', 'backbone', 'copy']):
        for form in ('inplace', 'dbbuf'):
            bad, where = 0, []
            for r in range(REPS):
                torch.cuda.synchronize()
                noise(kind)
                if form == 'inplace':
                    _lib.call('sad_frontend_run', fe._plan, _lib.ptr(pcm), B, pcm.stride(0), 0, _lib.ptr(out),
                              _lib.stream_handle(DEV))
                    got, exp = [out], [ref]
                else:
                    _lib.call('sad_frontend_run', fe._plan, _lib.ptr(pcm), B, pcm.stride(0), _lib.ptr(db),
                              _lib.ptr(out), _lib.stream_handle(DEV))
                    got, exp = [db, out], [ref_db, ref_m2]
                torch.cuda.synchronize()
                if not all(torch.equal(a, b) for a, b in zip(got, exp)):
                    bad += 1
                    d = got[0] != exp[0]
                    idx = d.nonzero()
                    if form == 'dbbuf' and DUMP:
                        # the wrong dB column(s) and the segment's PCM, for the bin attribution on the CPU
                        for sg, _, fr in idx[:4].tolist():
                            import numpy as np
                            np.savez(os.path.join(DUMP, f'fe_fail_{kind}_{r}_{sg}_{fr}.npz'), seg=sg, frame=fr,
                                     got=db[sg, :, fr].cpu().numpy(), ref=ref_db[sg, :, fr].cpu().numpy(),
                                     pcm=pcm[sg].cpu().numpy())
                    segs = sorted(set(idx[:, 0].tolist()))
                    s0 = segs[0]
                    fr = sorted(set(idx[idx[:, 0] == s0][:, 2].tolist()))
                    mel = sorted(set(idx[idx[:, 0] == s0][:, 1].tolist()))
                    where.append(f'{int(d.sum())} values, {len(segs)} segs {segs[:4]}; seg {s0}: {len(mel)} mels '
                                 f'{mel[:6]}, {len(fr)} frames {fr[:6]}, max |d| '
                                 f'{(got[0] - exp[0]).abs().max().item():.3g}')
            print(f'{kind:9s} {form:8s}: {bad:2d} of {REPS} differ' + ('' if not where else '; e.g. ' + where[0]),
                  flush=True)
            for w in where[1:4]:
                print(f'{"":20s}{w}', flush=True)


if __name__ == '__main__':
    main()
