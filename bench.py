#!/usr/bin/env python3
"""Headline benchmark: 4 s @ 32 kHz segments/sec end-to-end (mel + ResNet-18 +
6-head ensemble) on 1..8 MI355X, one process per GPU.

Workload per step and rank (BASELINE.json configs[1]+[2] combined): B = 2048
synthetic int16 segments already resident in HBM (generated on device by the
counter-hash PRNG, rank-disjoint ranges) -> fused STFT/mel/dB/standardise ->
fused resize+stem -> ResNet-18 (bf16 MFMA implicit GEMM) -> 6 heads + merge ->
RCCL all-gather of the merged logits to every rank (N > 1).  Weak scaling.

Prints ONE JSON line on rank 0 (driver contract) with `roofline` (the dominant
kernel, the 256x256 block-conv of layer3/4, MFMA-bound: algorithmic FLOPs of its
launches in the last timed step over their HIP-event durations recorded by
libsad on the launch stream; `traffic` from the committed PMC passes; the whole
backbone's rate as `roofline.backbone`) and `cpu_baseline` (the CPU oracle in the
reference's structure, on a bounded sample, rank 0 at N=1 only).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, 'synthetic-audio-detection_amd')
sys.path[:0] = [ROOT, PKG]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

SEG = 128000
# Algorithmic work per segment (DESIGN.md "Roofline accounting"):
BACKBONE_FLOP = 18.13e9        # ResNet-18 @512^2 with conv1's 3 identical channels folded (reference: 18.95e9)
REF_BACKBONE_FLOP = 18.95e9
BF16_PEAK_TFLOPS = 2500.0       # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
# The dominant kernel (36% of the step, profiles/r01_bench_kernels_final.md) and its
# rocprof key in profiles/r01_pmc_traffic.json; 1344 TFLOP/s = the best bf16 GEMM
# measured on this box (tools/gemm_ref.py)
DOMINANT_VARIANT = 13
DOMINANT_KERNEL = 'sad::block_conv_kernel<unsigned short, 2, 4, 8, 4, 2, 1, false>|131072'
# the same kernel's name in profiles taken before the epilogue-residual template flag (identical ISA)
DOMINANT_KERNEL_OLD = 'sad::block_conv_kernel<unsigned short, 2, 4, 8, 4, 2, 1>|131072'
F32_PEAK_TFLOPS = 157.3
FE_FLOP = 16.4e6               # per segment: window, rFFT 2.5 N log2 N x 251, |X|^2, mel, dB, stats
FE_BYTES = 256000 + 128512     # int16 PCM read + fp32 [128, 251] map written


def cpu_baseline(seconds: float = 15.0):
    """The reference's CPU path (oracle restatement, fp32, torch CPU): per-window
    front end, batch of up to 128 windows, ONE sub-model forward (configs[0])."""
    import numpy as np
    from oracle import frontend as ofe
    from oracle import resnet as ores
    from sad import weights as sw
    from sad.synth import synth_segment
    sd = sw.merged_state_dict(0, 1, False, bn_stats=sw.load_bn_stats(os.path.join(ROOT, 'tests', 'golden',
                                                                                    'bn_stats_n6.npz')))
    model = ores.load_merged_state(sd)
    cfg = ofe.SpectrogramConfig()
    pcm = [torch.from_numpy(synth_segment(0, i).astype(np.float32) / 32768.0) for i in range(8)]
    done, t0 = 0, time.perf_counter()
    with torch.no_grad():
        while time.perf_counter() - t0 < seconds:
            specs = torch.cat([ofe.waveform_to_spectrogram(w, 32000, cfg) for w in pcm])
            model(specs)
            done += len(pcm)
    dt = time.perf_counter() - t0
    return {'value': done / dt, 'unit': 'segments/s', 'cores': torch.get_num_threads(), 'kind': 'port',
            'sample': f'{done} synthetic 4 s segments in batches of 8 through the CPU oracle '
                      f'(per-window mel/dB/std/resize + 1 sub-model ResNet-18, fp32), {dt:.1f} s'}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--batch', type=int, default=2048, help='segments per GPU per step')
    ap.add_argument('--heads', type=int, default=6)
    ap.add_argument('--dtype', default='bf16', choices=['bf16', 'bf16x3', 'fp32'])
    ap.add_argument('--micro-batch', type=int, default=512,
                    help='segments per backbone launch sequence (stem/layer1/layer2 run in sub-batches of '
                         'SAD_FRONT_MB=32, layer3/4 on the whole micro-batch)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    args = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    if world > 1:
        dist.init_process_group('nccl', device_id=dev)

    from sad import _lib
    from sad import weights as sw
    from sad.engine import Engine
    stats = sw.load_bn_stats(os.path.join(ROOT, 'tests', 'golden', 'bn_stats_n6.npz'))
    sd = sw.merged_state_dict(0, args.heads, False, bn_stats=stats)
    eng = Engine(sd, dev, dtype=args.dtype, micro_batch=args.micro_batch)
    B = args.batch
    pcm = torch.empty(B, SEG, dtype=torch.int16, device=dev)
    _lib.call('sad_synth_pcm', 0, rank * B, B, SEG, _lib.ptr(pcm), _lib.stream_handle(dev))
    maps = torch.empty(B, 128, 251, device=dev)
    feats = torch.empty(B, 512, device=dev)
    logits = torch.empty(B, args.heads, 2, device=dev)
    merged = torch.empty(B, args.heads + 1, device=dev)
    gathered = torch.empty(world * B, args.heads + 1, device=dev) if world > 1 else None
    ev, fev = [], []

    def step(timed):
        if timed:
            f0, f1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            f0.record()
        m = eng.frontend(pcm)
        if timed:
            f1.record()
            fev.append((f0, f1))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        eng.backbones[0](m, out=feats)
        if timed:
            e1.record()
            ev.append((e0, e1))
        eng.heads([feats], logits, merged)
        if gathered is not None:
            dist.all_gather_into_tensor(gathered, merged)

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if i == args.steps - 1:
            # HIP events around each block-conv launch of the last timed step, on
            # its stream (events between launches cost the step ~5%, so one step only)
            _lib.call('sad_profile_begin')
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    k_ms, k_n, k_fl = _lib.ctypes.c_double(), _lib.I64(), _lib.ctypes.c_double()
    _lib.call('sad_profile_end', DOMINANT_VARIANT, _lib.ctypes.byref(k_ms), _lib.ctypes.byref(k_n),
              _lib.ctypes.byref(k_fl))
    bb_ms = sum(a.elapsed_time(b) for a, b in ev) / len(ev)
    fe_ms = sum(a.elapsed_time(b) for a, b in fev) / len(fev)
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    ms = elapsed * 1e3 / args.steps
    value = world * B * args.steps / elapsed
    if rank == 0:
        peak = BF16_PEAK_TFLOPS if args.dtype == 'bf16' else F32_PEAK_TFLOPS
        achieved = BACKBONE_FLOP * B / (bb_ms * 1e-3) / 1e12
        n_l = max(k_n.value, 1)
        k_avg_us = k_ms.value * 1e3 / n_l
        k_tf = k_fl.value / (k_ms.value * 1e-3) / 1e12 if k_ms.value > 0 else 0.0
        traffic = None
        tj = os.path.join(ROOT, 'profiles', 'r01_pmc_traffic.json')
        if os.path.exists(tj) and args.dtype == 'bf16':
            tr = json.load(open(tj))
            rec = tr.get(DOMINANT_KERNEL) or tr.get(DOMINANT_KERNEL_OLD)
            if rec and rec.get('hbm_read_bytes') is not None:
                traffic = rec['hbm_read_bytes'] + rec['hbm_write_bytes']
        out = {
            'metric': '4s@32kHz segments/sec end-to-end (mel+ResNet+ensemble), 1/2/4/8 MI355X',
            'value': round(value, 1), 'unit': 'segments/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(ms, 3), 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': args.dtype,
            'data': 'synthetic int16 PCM (counter-hash PRNG, generated in HBM) + random-init ResNet-18/6 heads '
                    '(hash PRNG, BN-calibrated)',
            'config': {'workload': 'end-to-end inference: B int16 4 s segments resident in HBM -> mel front end '
                                   '-> ResNet-18@512x512 -> 6 binary heads -> merge (+RCCL all-gather of logits)',
                       'segments_per_gpu_per_step': B, 'heads': args.heads, 'distinct_backbones': 1,
                       'micro_batch': args.micro_batch, 'parallelism': f'dp{world}'},
            'roofline': {'bound': 'mfma',
                         'kernel': 'sad::block_conv_kernel 256x256 tile (variant 13): the layer3 + layer4 convs, '
                                   '8 launches per micro-batch, about 35% of the step',
                         'achieved': round(k_tf, 1), 'peak': peak, 'unit': 'TFLOP/s', 'frac': round(k_tf / peak, 4),
                         'traffic': traffic, 'traffic_unit': 'HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE, '
                                                             'profiles/r01_pmc_traffic.json)',
                         'launches': k_n.value, 'launch_avg_us': round(k_avg_us, 2),
                         'flop_per_launch': round(k_fl.value / n_l),
                         'backbone': {'achieved': round(achieved, 1), 'frac': round(achieved / peak, 4),
                                      'ms_per_step': round(bb_ms, 3), 'flop_per_segment': BACKBONE_FLOP,
                                      'what': 'fused resize+stem + 16 block-conv GEMMs + avgpool, HIP events '
                                              'around the backbone call'},
                         'measured_gemm_ceiling_tflops': 1344.0,
                         # front end (configs[1]): fused STFT/mel/dB + standardise, fp32 VALU-bound
                         # (16.4 MFLOP and 384,512 B per segment)
                         'frontend': {'ms_per_step': round(fe_ms, 3),
                                      'achieved_tflops': round(FE_FLOP * B / (fe_ms * 1e-3) / 1e12, 2),
                                      'peak_tflops': F32_PEAK_TFLOPS,
                                      'frac': round(FE_FLOP * B / (fe_ms * 1e-3) / 1e12 / F32_PEAK_TFLOPS, 4),
                                      'achieved_gbps': round(FE_BYTES * B / (fe_ms * 1e-3) / 1e9, 1),
                                      'segments_per_s': round(B / (fe_ms * 1e-3), 1)}},
        }
        if world == 1 and not args.no_cpu_baseline:
            out['cpu_baseline'] = cpu_baseline()
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
