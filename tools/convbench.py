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
    args = ap.parse_args()
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


if __name__ == '__main__':
    main()
