#!/usr/bin/env python3
"""Diagnostic: per-phase cycle stamps of workgroup 0 (waves 0 and NW/2) for the
layer1 halo kernel (variant 25) and the 256x256 block conv (variant 13), from
a -DSAD_STAMPS=1 build of libsad (SAD_LIB=abl/libsad_stamps.so):

    make -C synthetic-audio-detection_amd/csrc OUT=$PWD/abl/libsad_stamps.so BUILD=/tmp/stampobj \\
        CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -DSAD_STAMPS=1"
    SAD_LIB=abl/libsad_stamps.so python tools/stamp_conv.py

The library prints one line per launch and wave to stderr.  Variant 25 phases
per tile: 0-1 taps issued, 1-2 epilogue (early waves) / wait, 2-3 tile barrier,
3-next late epilogue.  Variant 13 per K-step: wait+barrier, reads+DMA, MFMA
issue, tail.  Stamping costs about 11 % of wave cycles.

The same build also stamps (s_memtime, s_memrealtime) at entry and exit of
wave 0 of every workgroup and prints the in-kernel clock (median and per XCD),
the launch span and the spread of workgroup end times.  For the clock under
load, stamp every n-th launch inside the bench loop instead:

    SAD_LIB=abl/libsad_stamps.so SAD_STAMP_EVERY=1000 python bench.py --kernels-only --steps 300"""
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
    # the bench's Infinity-Cache-sized sub-batch (32 images: 8 tiles per workgroup)
    # and 512 images (128 tiles per workgroup, operands from HBM)
    w = rnd((64, 576), 3, (2 / 576) ** 0.5)
    b = torch.zeros(64, device=DEV)
    for n in (32, 512):
        x = rnd((n, 128, 128, 64), 1)
        res = rnd((n, 128, 128, 64), 2)
        for name, kw in (('layer1 conv (v25)', {}), ('layer1 conv + res (v25)', {'res': res})):
            for it in range(3):
                print(f'--- {name}, {n} images, iteration {it}', file=sys.stderr, flush=True)
                block_conv(x, w, b, 1, 1, variant=25, **kw)
                torch.cuda.synchronize()
    x4 = rnd((256, 16, 16, 512), 4)
    w4 = rnd((512, 4608), 5, (2 / 4608) ** 0.5)
    b4 = torch.zeros(512, device=DEV)
    for it in range(3):
        print(f'--- layer4 conv2 (v13), 256 images, iteration {it}', file=sys.stderr, flush=True)
        block_conv(x4, w4, b4, 1, 1, variant=13)
        torch.cuda.synchronize()


if __name__ == '__main__':
    main()
