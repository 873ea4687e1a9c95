#!/usr/bin/env python3
"""Throughput of the deeper timm backbones on one GPU:
synthetic int16 PCM resident in HBM -> front end -> resnet34/50/101/152 (generic
libsad ResNet plan) -> N heads -> merge.  Not the driver's bench line (that is
bench.py, ResNet-18); prints one JSON line per architecture.

  python tools/bench_arch.py --arch resnet50 resnet34 --batch 512 --steps 5
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'synthetic-audio-detection_amd'))

import torch  # noqa: E402

SEG = 128000
BF16_PEAK_TFLOPS = 2500.0


def backbone_flop(name: str) -> float:
    """Algorithmic FLOPs per 512x512 segment: 2 * MACs of every conv (stem at
    256x256 output, maxpool to 128x128, then the stages)."""
    from sad import weights as sw
    block, layers, _ = sw.arch_spec(name)
    fl = 2.0 * 256 * 256 * 64 * 3 * 49
    H, inp = 128, 64
    for li, (planes, n) in enumerate(zip(sw.BLOCK_CHANNELS, layers)):
        for b in range(n):
            s = 2 if (b == 0 and li > 0) else 1
            Ho = H // s
            if block == 'bottleneck':
                cout = planes * 4
                fl += 2.0 * (H * H * planes * inp + Ho * Ho * planes * planes * 9 + Ho * Ho * cout * planes)
            else:
                cout = planes
                fl += 2.0 * (Ho * Ho * planes * inp * 9 + Ho * Ho * planes * planes * 9)
            if b == 0 and (s != 1 or inp != cout):
                fl += 2.0 * Ho * Ho * cout * inp
            H, inp = Ho, cout
    return fl


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--arch', nargs='+', default=['resnet50'])
    ap.add_argument('--batch', type=int, default=512)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--heads', type=int, default=6)
    ap.add_argument('--micro-batch', type=int, default=64)
    ap.add_argument('--dtype', default='bf16', choices=['bf16', 'bf16x3', 'fp32'])
    args = ap.parse_args()
    from sad import _lib
    from sad import weights as sw
    from sad.engine import Engine
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    B = args.batch
    pcm = torch.empty(B, SEG, dtype=torch.int16, device=dev)
    _lib.call('sad_synth_pcm', 0, 0, B, SEG, _lib.ptr(pcm), _lib.stream_handle(dev))
    for name in args.arch:
        eng = Engine(sw.merged_state_dict(0, args.heads, False, model_name=name), dev, args.dtype,
                     args.micro_batch)
        ev = []

        def step(timed):
            m = eng.frontend(pcm)
            if timed:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
            f = eng.backbones[0](m)
            if timed:
                e1.record()
                ev.append((e0, e1))
            return eng.heads([f])

        for _ in range(args.warmup):
            step(False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            _, merged = step(True)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        bb_ms = sum(a.elapsed_time(b) for a, b in ev) / len(ev)
        fl = backbone_flop(name)
        tf = fl * B / (bb_ms * 1e-3) / 1e12
        print(json.dumps({'arch': name, 'segments_per_s': round(B * args.steps / el, 1), 'batch': B,
                          'heads': args.heads, 'micro_batch': eng.backbones[0].micro_batch, 'dtype': args.dtype,
                          'backbone_ms_per_step': round(bb_ms, 3), 'backbone_gflop_per_segment': round(fl / 1e9, 3),
                          'backbone_tflops': round(tf, 1), 'frac_of_bf16_peak': round(tf / BF16_PEAK_TFLOPS, 4),
                          'finite': bool(torch.isfinite(merged).all().item())}), flush=True)
        del eng
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
