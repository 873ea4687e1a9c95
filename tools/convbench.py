#!/usr/bin/env python3
"""Tile-variant sweep for the implicit-GEMM conv kernel over ResNet-18's layer
shapes (bf16).  Prints one line per (shape, micro-batch, variant) with the
median kernel time and TFLOP/s; checks that every variant's output is
bitwise identical to variant 1's (same K order per output element).

    python tools/convbench.py [--mb 16 32 64 128] [--variants 1 2 3 ...]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'synthetic-audio-detection_amd')]

import torch  # noqa: E402

from sad.engine import conv2d  # noqa: E402

# name, H(in), Cin, Cout, k, stride, pad, residual
SHAPES = [
    ('l1.conv', 128, 64, 64, 3, 1, 1, True),
    ('l2.c1', 128, 64, 128, 3, 2, 1, False),
    ('l2.c2', 64, 128, 128, 3, 1, 1, True),
    ('l2.ds', 128, 64, 128, 1, 2, 0, False),
    ('l3.c1', 64, 128, 256, 3, 2, 1, False),
    ('l3.c2', 32, 256, 256, 3, 1, 1, True),
    ('l3.ds', 64, 128, 256, 1, 2, 0, False),
    ('l4.c1', 32, 256, 512, 3, 2, 1, False),
    ('l4.c2', 16, 512, 512, 3, 1, 1, True),
    ('l4.ds', 32, 256, 512, 1, 2, 0, False),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--mb', type=int, nargs='+', default=[32, 64, 128])
    ap.add_argument('--variants', type=int, nargs='+', default=[1, 2, 3, 4, 5, 6, 7, 8])
    ap.add_argument('--iters', type=int, default=10)
    ap.add_argument('--shapes', nargs='*', default=None)
    ap.add_argument('--blocks', action='store_true', help='sweep the block-conv kernels (variants 9-18, 20)')
    ap.add_argument('--ablate', type=int, nargs='+', default=[0], help='block kernel timing ablations (bit mask)')
    ap.add_argument('--split', action='store_true', help='split-bf16 (bf16x3) operands; FLOP/s count 3 MFMA '
                                                         'products per MAC in the "exec" column')
    args = ap.parse_args()
    if args.blocks:
        bench_blocks(args.mb, [v for v in args.variants if v >= 9] or list(range(9, 19)) + [20], args.iters, args.shapes,
                     tuple(args.ablate), args.split)
        return
    dev = torch.device('cuda:0')
    torch.manual_seed(0)
    for name, H, Cin, Cout, k, s, p, res in SHAPES:
        if args.shapes and name not in args.shapes:
            continue
        Ho = (H + 2 * p - k) // s + 1
        w = (torch.randn(Cout, k, k, Cin, device=dev) * (2.0 / (k * k * Cin)) ** 0.5).to(torch.bfloat16)
        bias = torch.randn(Cout, device=dev) * 0.1
        for mb in args.mb:
            x = torch.randn(mb, H, H, Cin, device=dev).to(torch.bfloat16)
            r = torch.randn(mb, Ho, Ho, Cout, device=dev).to(torch.bfloat16) if res else None
            flop = 2.0 * mb * Ho * Ho * Cout * k * k * Cin
            ref = None
            for v in args.variants:
                if Cout % 128 and v in (3, 4, 5, 8):
                    continue
                out = torch.empty(mb, Ho, Ho, Cout, device=dev, dtype=torch.bfloat16)
                try:
                    conv2d(x, w, bias, s, p, r, True, v, out)
                except RuntimeError as e:
                    print(f'{name:8s} mb={mb:4d} v={v}: {e}')
                    continue
                torch.cuda.synchronize()
                same = 'ref'
                if ref is None:
                    ref = out.clone()
                else:
                    same = 'same' if torch.equal(out, ref) else f'DIFF {(out.float() - ref.float()).abs().max().item():.3g}'
                ts = []
                for _ in range(args.iters):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    conv2d(x, w, bias, s, p, r, True, v, out)
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1))
                ts.sort()
                t = ts[len(ts) // 2]
                print(f'{name:8s} mb={mb:4d} v={v}: {t * 1e3:9.1f} us  {flop / t / 1e9:7.1f} TF/s  {same}', flush=True)


BLOCKS = [  # name, H(in), Cin, Cout, stride, shortcut
    ('l1.c2+id', 128, 64, 64, 1, 'id'),
    ('l1.c1', 128, 64, 64, 1, None),
    ('l2.c1', 128, 64, 128, 2, None),
    ('l2.c2+ds', 64, 128, 128, 1, 'ds'),
    ('l2.c2+id', 64, 128, 128, 1, 'id'),
    ('l2.c1b', 64, 128, 128, 1, None),
    ('l3.c1', 64, 128, 256, 2, None),
    ('l3.c2+ds', 32, 256, 256, 1, 'ds'),
    ('l3.c2+id', 32, 256, 256, 1, 'id'),
    ('l4.c1', 32, 256, 512, 2, None),
    ('l4.c2+ds', 16, 512, 512, 1, 'ds'),
    ('l4.c2+id', 16, 512, 512, 1, 'id'),
]


def bench_blocks(mbs, variants, iters, shapes=None, ablate=(0,), split=False):
    from sad.engine import block_conv, to_split
    dev = torch.device('cuda:0')
    cvt = (lambda t: to_split(t.float())) if split else (lambda t: t)
    for name, H, Cin, Cout, s, sc in BLOCKS:
        if shapes and name not in shapes:
            continue
        Ho = H // s
        cin0 = Cin if sc is None else Cout
        h0 = H if sc is None else Ho
        cin1 = Cout // 2  # the downsample reads the previous stage's map (Cout/2 channels, 2x the side)
        K = 9 * cin0 + (0 if sc is None else (Cout if sc == 'id' else cin1))
        w = cvt((torch.randn(Cout, K, device=dev) * (1.0 / K) ** 0.5).to(torch.bfloat16))
        bias = torch.randn(Cout, device=dev) * 0.1
        for mb in mbs:
            x = cvt(torch.randn(mb, h0, h0, cin0, device=dev).to(torch.bfloat16))
            scx = None
            if sc == 'id':
                scx = cvt(torch.randn(mb, Ho, Ho, Cout, device=dev).to(torch.bfloat16))
            elif sc == 'ds':
                scx = cvt(torch.randn(mb, 2 * Ho, 2 * Ho, cin1, device=dev).to(torch.bfloat16))
            stride = s if sc is None else 1
            flop = 2.0 * mb * Ho * Ho * Cout * K
            ref = None
            bc = {9: 64, 10: 128, 11: 64, 12: 128, 13: 256, 14: 128, 15: 128, 16: 64, 17: 256, 18: 128, 20: 64, 21: 64, 25: 64, 30: 256, 31: 256, 32: 128, 41: 128, 42: 64, 43: 128, 44: 128}
            for v0 in [v + (ab << 8) for v in variants for ab in ablate]:
                v = v0 & 255
                if Cout % bc[v] or (v in (20, 21, 25) and (stride != 1 or sc == 'ds')) or (v == 25 and Cout != 64) or \
                        (v in (30, 31) and (stride != 1 or Ho % 16)) or (v in (32, 44) and (stride != 2 or Ho % 16)) or \
                        (v == 41 and (stride != 1 or Cout != 128 or sc == 'id')) or \
                        (v == 42 and (stride != 1 or Cout != 64 or sc == 'ds' or not split)) or \
                        (v == 43 and (stride != 2 or Cin != 64 or Cout != 128 or Ho % 16)):
                    continue
                # the halo kernel (20) takes the identity shortcut as an epilogue residual
                kw = dict(res=scx) if v in (20, 21, 25, 42) else dict(sc=scx, sc_stride=2 if sc == 'ds' else 1)
                if sc == 'id' and v == 13 and (v0 >> 8) & 512:
                    kw = dict(res=scx)  # ablate bit 512: the identity as the epilogue residual (RES)

                def run(o=None):
                    return block_conv(x, w, bias, stride, 1, relu=True, variant=v0, out=o, split=split, **kw)
                out = run()
                torch.cuda.synchronize()
                same = 'ref' if ref is None else ('same' if torch.equal(out, ref) else
                                                  f'DIFF {(out.float() - ref.float()).abs().max().item():.3g}')
                ref = out.clone() if ref is None else ref
                # steady state: warm-up launches, then 3 timed runs of `iters`
                # back-to-back launches each (per-launch events with a sync between
                # launches let the clock drop and gave ~6 % run-to-run noise)
                for _ in range(3):
                    run(out)
                ts = []
                for _ in range(3):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(iters):
                        run(out)
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) / iters)
                ts.sort()
                t = ts[1]
                ex = f'  exec {3 * flop / t / 1e9:7.1f} TF/s' if split else ''
                print(f'{name:9s} mb={mb:4d} v={v} ablate={v0 >> 8}: {t * 1e3:9.1f} us  {flop / t / 1e9:7.1f} TF/s{ex}  '
                      f'{same}', flush=True)


if __name__ == '__main__':
    main()
