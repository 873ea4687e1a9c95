"""Locate front-end disagreements vs the oracle over a 1,024-segment synthetic
batch (seed 11): per segment max|d map|, and for the worst ones where it sits
(mel bin, frame), the dB values, the segment's max / mean / std on both sides."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'synthetic-audio-detection_amd')]
from oracle import frontend as ofe  # noqa: E402
from sad import _lib  # noqa: E402
from sad.engine import FrontEnd  # noqa: E402

DEV = 'cuda:0'
n = 1024
pcm = torch.empty(n, 128000, dtype=torch.int16, device=DEV)
_lib.call('sad_synth_pcm', 11, 0, n, 128000, _lib.ptr(pcm), _lib.stream_handle(torch.device(DEV)))
m, db = FrontEnd(DEV)(pcm, want_db=True)
torch.cuda.synchronize()
host, dm, ddb = pcm.cpu(), m.cpu(), db.cpu()
per = []
for s in range(0, n, 128):
    rdb, ref = ofe.batch_maps(host[s:s + 128])
    d = (dm[s:s + 128] - ref).abs().amax(dim=(1, 2))
    e = (ddb[s:s + 128] - rdb).abs().amax(dim=(1, 2))
    for i in range(128):
        per.append((d[i].item(), e[i].item(), s + i))
per.sort(reverse=True)
print('worst segments (max|d map|, max|d dB|, idx):', per[:12])
print('segments over 2e-4:', sum(1 for p in per if p[0] > 2e-4))
np.save('gpurun_out/fe_diag_idx.npy', np.array([p[2] for p in per[:8]]))
for dmx, dbx, i in per[:4]:
    rdb, ref = ofe.batch_maps(host[i:i + 1])
    a, b = dm[i], ref[0]
    k = (a - b).abs().argmax().item()
    mb, fr = divmod(k, a.shape[1])
    da, db_ = ddb[i], rdb[0]
    print(f'seg {i}: at mel {mb} frame {fr}: dev map {a[mb, fr]:.6f} ref {b[mb, fr]:.6f}; '
          f'dev dB {da[mb, fr]:.6f} ref dB {db_[mb, fr]:.6f}')
    print(f'   dB max dev {da.max():.6f} ref {db_.max():.6f}; clamp floor dev {da.max() - 80:.6f}')
    print(f'   frac at floor dev {(da <= da.max() - 80 + 1e-6).float().mean():.4f} ref {(db_ <= db_.max() - 80 + 1e-6).float().mean():.4f}')
    print(f'   dB mean dev {da.double().mean():.6f} ref {db_.double().mean():.6f}; std dev {da.double().std():.6f} ref {db_.double().std():.6f}')
    print(f'   max|d dB| {((da - db_).abs().max()):.3e} at {divmod((da - db_).abs().argmax().item(), a.shape[1])}')
    print(f'   pcm absmax {host[i].abs().max().item()} std {host[i].float().std():.2f}')
