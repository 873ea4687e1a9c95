#!/usr/bin/env python3
"""Diagnostic: per-K-step phase stamps (waves 0 and 4 of workgroup 0) of the
layer4 conv2 shape on variant 13 (implicit GEMM) and variant 30 (patch-resident
256 x 256), from a -DSAD_STAMPS=1 build (SAD_LIB=abl/libsad_stamps.so; see
tools/stamp_conv.py).  Phases: 0-1 wait + barrier, 1-2 half-0 reads (+ the
weight waves' DMA issue), 2-3 MFMAs (+ the patch waves' DMA issue), 3-next tail."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'synthetic-audio-detection_amd')]

import torch  # noqa: E402

from sad.engine import block_conv  # noqa: E402

DEV = 'cuda:0'


def rnd(shape, seed, scale=1.0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return (torch.randn(shape, generator=g, device=DEV) * scale).to(torch.bfloat16)


def main():
    n = int(os.environ.get('STAMP_N', '256'))
    x4 = rnd((n, 16, 16, 512), 4)
    w4 = rnd((512, 4608 + 512), 5, (2 / 4608) ** 0.5)
    b4 = torch.zeros(512, device=DEV)
    sc = rnd((n, 16, 16, 512), 6)
    for v in (13, 30):
        for tag, kw in (('plain', {}), ('+id', {'sc': sc})):
            for it in range(2):
                print(f'--- layer4 conv2 {tag} (v{v}), {n} images, iteration {it}', file=sys.stderr, flush=True)
                block_conv(x4, w4, b4, 1, 1, variant=v, **kw)
                torch.cuda.synchronize()


if __name__ == '__main__':
    main()
