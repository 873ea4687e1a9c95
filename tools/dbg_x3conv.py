#!/usr/bin/env python3
"""Error map of a split-bf16 3x3 conv variant against float64 (debugging aid):
where (channel, tile row, tile column, image) the relative error sits.
    python tools/dbg_x3conv.py --variant 42 [--res] [--H 32] [--N 2]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'synthetic-audio-detection_amd')]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--variant', type=int, default=42)
    ap.add_argument('--res', action='store_true')
    ap.add_argument('--H', type=int, default=32)
    ap.add_argument('--N', type=int, default=2)
    ap.add_argument('--c', type=int, default=64)
    ap.add_argument('--zero-lo', action='store_true', help='inputs and weights exact in bf16 (lo = 0)')
    args = ap.parse_args()
    from sad.engine import block_conv, from_split, to_split
    g = torch.Generator().manual_seed(1)
    N, H, c = args.N, args.H, args.c
    x = torch.randn(N, H, H, c, generator=g).clamp_min(0)
    r = torch.randn(N, H, H, c, generator=g).clamp_min(0) if args.res else None
    w = torch.randn(c, c, 3, 3, generator=g) * (2.0 / (9 * c)) ** 0.5
    if args.zero_lo:
        x = x.to(torch.bfloat16).float()
        w = w.to(torch.bfloat16).float()
        r = r.to(torch.bfloat16).float() if r is not None else None
    bias = torch.randn(c, generator=g) * 0.1
    y = F.conv2d(x.permute(0, 3, 1, 2).double(), w.double(), bias.double(), padding=1).permute(0, 2, 3, 1)
    ref = (y + (r.double() if r is not None else 0)).clamp_min(0)
    wk = w.permute(0, 2, 3, 1).reshape(c, 9 * c)
    out = block_conv(to_split(x).cuda(), to_split(wk).cuda(), bias.cuda(), variant=args.variant, split=True,
                     res=to_split(r).cuda() if r is not None else None)
    torch.cuda.synchronize()
    got = from_split(out.cpu()).double()
    e = (got - ref).abs() / ref.abs().max()
    print(f'v{args.variant} res={args.res} zero_lo={args.zero_lo}: max rel {e.max():.3e}')
    # by channel (groups of 4), by tile row-in-tile, column-in-tile, image
    ch = e.amax(dim=(0, 1, 2))
    print('per channel max (x1e-4):', [round(v * 1e4, 2) for v in ch.tolist()])
    rows = e.amax(dim=(0, 2, 3)).view(-1, 16).amax(0)
    print('per row-in-tile max (x1e-4):', [round(v * 1e4, 2) for v in rows.tolist()])
    cols = e.amax(dim=(0, 1, 3)).view(-1, 16).amax(0)
    print('per column-in-tile max (x1e-4):', [round(v * 1e4, 2) for v in cols.tolist()])
    print('per image max (x1e-4):', [round(v * 1e4, 2) for v in e.amax(dim=(1, 2, 3)).tolist()])
    bad = (e > 1e-4).nonzero()
    print('outputs above 1e-4:', bad.shape[0], 'of', e.numel(), '; first:', bad[:8].tolist())
    # hi part alone vs bf16(ref)
    raw = out.cpu().view(N, H, H, -1, 2, 32)
    hi = raw[:, :, :, :, 0, :].reshape(N, H, H, c).float().double()
    print(f'hi vs ref: max rel {((hi - ref).abs() / ref.abs().max()).max():.3e} (bf16 rounding ~2e-3)')


if __name__ == '__main__':
    main()
