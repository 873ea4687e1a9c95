#!/usr/bin/env python3
"""BASELINE.json configs[3]: batched inference over a shard of 1,000,000
synthetic 4 s segments, one process per GPU, ONE RCCL all-gather of the merged
logits at the end.

Each rank takes the contiguous range shard_range(n, rank, world) of the global
segment ids; segments are generated on the device in chunks by the counter-hash
PRNG (sad_synth_pcm, keyed by the GLOBAL segment id, so the result does not
depend on the world size) -- generation is timed separately and excluded from
the inference rate, as SURVEY 8(d) prescribes.  Prints one JSON line on rank 0.

    python tools/run_1m.py [--gpus N] [--total 1000000] [--chunk 4096] [--host-fed] [--dtype bf16x3]
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/run_1m.py --gpus 8

``--gpus N`` without a launcher starts the N ranks itself (sad/launch.py); under
a launcher the world size must equal N.

--host-fed (SURVEY 8(d) "host-fed (pinned H2D) variant"): each chunk's int16
PCM is copied from pinned host memory on the compute stream, before its
inference (round 4 overlapped the copy on a side stream; round 5 dropped
cross-stream hand-offs); the rate is wall-clock over the whole
loop, PCIe included.  The host source is a ring of 2 pinned chunks
(filled once, before timing) -- 1 M segments are 256 GB -- so the logits
repeat with the ring and their checksum differs from the device-synth mode.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'synthetic-audio-detection_amd')]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

SEG = 128000


def main(argv=None, return_logits: bool = False):
    """Runs the shard; with ``return_logits`` (in-process callers, e.g. the GPU
    test) returns (the JSON record, gathered merged logits on the CPU) on rank 0."""
    ap = argparse.ArgumentParser()
    ap.add_argument('--total', type=int, default=1_000_000)
    ap.add_argument('--chunk', type=int, default=4096, help='segments per device batch')
    ap.add_argument('--heads', type=int, default=6)
    ap.add_argument('--dtype', default='bf16', choices=['bf16', 'bf16x3', 'fp32'])
    ap.add_argument('--micro-batch', type=int, default=0, help='0: 2048 bf16, 512 bf16x3, 128 fp32 (as bench.py)')
    ap.add_argument('--host-fed', action='store_true', help='PCM from pinned host memory (H2D inside the timing)')
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--backend', default='nccl', choices=['nccl', 'gloo'], help='gloo: tests only')
    ap.add_argument('--one-device', action='store_true', help='every rank on cuda:0 (2-rank test on one GPU)')
    ap.add_argument('--out-logits', default='', help='rank 0 saves the gathered logits here (tests)')
    args = ap.parse_args(argv)
    args.micro_batch = args.micro_batch or {'bf16': 2048, 'bf16x3': 512, 'fp32': 128}[args.dtype]

    from sad import launch
    if args.gpus > 1 and not launch.under_launcher():
        rc = launch.relaunch(args.gpus, os.path.abspath(__file__), sys.argv[1:] if argv is None else list(argv))
        if argv is None:
            sys.exit(rc)
        return rc
    world, rank, local = launch.check_world(args.gpus)
    dev = torch.device('cuda', 0 if args.one_device else local)
    torch.cuda.set_device(dev)
    if world > 1:
        if args.backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
        else:
            dist.init_process_group('gloo')

    from sad import _lib
    from sad import weights as sw
    from sad.distributed import gather_rows, shard_range
    from sad.engine import Engine
    stats = sw.load_bn_stats(os.path.join(ROOT, 'tests', 'golden', 'bn_stats_n6.npz'))
    eng = Engine(sw.merged_state_dict(0, args.heads, False, bn_stats=stats), dev, dtype=args.dtype,
                 micro_batch=args.micro_batch)
    s, e = shard_range(args.total, rank, world)
    pcm = torch.empty(args.chunk, SEG, dtype=torch.int16, device=dev)
    local_out = torch.empty(e - s, args.heads + 1, device=dev)
    stream = _lib.stream_handle(dev)

    # warm-up (plans, workspaces) on the first chunk, untimed
    _lib.call('sad_synth_pcm', 0, s, min(args.chunk, e - s), SEG, _lib.ptr(pcm), stream)
    eng.forward_pcm(pcm[:min(args.chunk, e - s)])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()

    gen_s = inf_s = 0.0
    g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    i0, i1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if args.host_fed:
        ring = []
        for k in range(2):
            n = min(args.chunk, e - s)
            _lib.call('sad_synth_pcm', 0, s + k * args.chunk, n, SEG, _lib.ptr(pcm), stream)
            h = torch.empty(args.chunk, SEG, dtype=torch.int16, pin_memory=True)
            h[:n].copy_(pcm[:n])
            ring.append(h)
        dbuf = [pcm, torch.empty_like(pcm)]
        starts = list(range(s, e, args.chunk))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for j, c in enumerate(starts):
            b, n = j % 2, min(args.chunk, e - c)
            # the copy runs on the compute stream: a copy stream's hand-off to
            # the front end is the cross-stream pattern bench.Mode dropped in
            # round 5
            dbuf[b][:n].copy_(ring[j % 2][:n], non_blocking=True)
            _, merged = eng.forward_pcm(dbuf[b][:n])
            local_out[c - s:c - s + n] = merged
        torch.cuda.synchronize()
        inf_s = time.perf_counter() - t0
    else:
        t0 = time.perf_counter()
    for c in (range(s, e, args.chunk) if not args.host_fed else []):
        n = min(args.chunk, e - c)
        g0.record()
        _lib.call('sad_synth_pcm', 0, c, n, SEG, _lib.ptr(pcm), stream)
        g1.record()
        i0.record()
        _, merged = eng.forward_pcm(pcm[:n])
        local_out[c - s:c - s + n] = merged
        i1.record()
        torch.cuda.synchronize()
        gen_s += g0.elapsed_time(g1) / 1e3
        inf_s += i0.elapsed_time(i1) / 1e3
    t_loop = time.perf_counter() - t0
    a0 = time.perf_counter()
    allz = gather_rows(local_out, args.total) if world > 1 else local_out
    torch.cuda.synchronize()
    t_gather = time.perf_counter() - a0
    if world > 1:
        t = torch.tensor([inf_s, t_loop, t_gather], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        inf_s, t_loop, t_gather = t.tolist()
    rec = None
    if rank == 0:
        finite = bool(torch.isfinite(allz).all().item())
        rec = {
            'metric': '4s@32kHz segments/sec end-to-end (mel+ResNet+ensemble), 1M-segment shard (configs[3])'
                      + (', host-fed (pinned H2D, PCIe-inclusive wall clock)' if args.host_fed else ''),
            'value': round(args.total / (inf_s + t_gather), 1), 'unit': 'segments/s', 'n_gpus': world,
            'total_segments': args.total, 'chunk': args.chunk, 'dtype': args.dtype,
            'inference_s_max_rank': round(inf_s, 3), 'allgather_s': round(t_gather, 4),
            'synthesis_s_rank0_excluded': round(gen_s, 3), 'wall_loop_s_max_rank': round(t_loop, 3),
            'gathered_rows': int(allz.shape[0]), 'all_finite': finite,
            'logits_checksum': round(float(allz.double().sum().item()), 3)}
        print(json.dumps(rec), flush=True)
        if args.out_logits:
            torch.save(allz.cpu(), args.out_logits)
    if world > 1:
        dist.destroy_process_group()
    if return_logits:
        return rec, allz.cpu()
    return rec


if __name__ == '__main__':
    main()
