#!/usr/bin/env python3
"""Headline benchmark: 4 s @ 32 kHz segments/sec end-to-end (mel + ResNet-18 +
6-head ensemble) on 1..8 MI355X, one process per GPU.

Workload per step and rank (BASELINE.json configs[1]+[2] combined): B = 2048
synthetic int16 segments already resident in HBM (generated on device by the
counter-hash PRNG, rank-disjoint ranges) -> fused STFT/mel/dB/standardise ->
fused resize+stem -> ResNet-18 (bf16 MFMA implicit GEMM) -> 6 heads + merge ->
RCCL all-gather of the merged logits to every rank (N > 1).  Weak scaling.

``--gpus N`` without a launcher starts N ranks itself (sad/launch.py: a
torch.distributed.run child); under a launcher the world size must equal N.

Prints ONE JSON line on rank 0 (driver contract).  Besides the headline (bf16,
configs[2]) it carries, measured in the same run on the same segments:
  * ``parity_mode``: the split-bf16 mode (dtype bf16x3) that meets the
    north-star |dlogit| <= 1e-3 -- its segments/s, roofline of its dominant
    kernel, max|dlogit| against the reference-generated golden logits and
    against the fp32 device path over the whole batch, decision agreement;
  * ``accuracy``: the same numbers for the bf16 headline mode;
  * ``fp32_mode``: the f32-MFMA mode's rate (N = 1);
  * ``roofline`` (the dominant kernel, variant 31 of the layer3/4 stride-1 convs:
    algorithmic FLOPs of its launches in the last timed step over their HIP
    event durations recorded by libsad on the launch stream; ``traffic`` from
    the committed PMC passes) and ``cpu_baseline`` (configs[0]: the CPU oracle
    in the reference's structure on 64 synthetic WAV clips, rank 0 at N = 1).
"""
import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, 'synthetic-audio-detection_amd')
sys.path[:0] = [ROOT, PKG]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from sad import launch  # noqa: E402

SEG = 128000
# Algorithmic work per segment:
BACKBONE_FLOP = 18.13e9        # ResNet-18 @512^2 with conv1's 3 identical channels folded (reference: 18.95e9)
BF16_PEAK_TFLOPS = 2500.0      # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
F32_PEAK_TFLOPS = 157.3        # f32 MFMA = f32 vector peak (MI355X_MICROARCH.md)
# The dominant kernel of each mode: (libsad profile variant, rocprof name prefix
# (every template instantiation is launch-weighted, see dominant_traffic, so a
# template change cannot make the key stale), what it is, the committed PMC
# traffic file of that mode written by tools/profile_bench.sh)
DOMINANT = {
    'bf16': (31, 'sad::halo256r_kernel<',
             'sad::halo256r_kernel (variant 31): patch-resident 256-channel x 16x16-pixel conv, weights streamed '
             'into registers; the stride-1 layer3/4 convs of a step (5 convs; layer3.0 conv2 + downsample runs as '
             'two image-range launches at micro-batch 2,048, the last one fuses the average pool)',
             ('r06_pmc_traffic.json', 'r05_pmc_traffic.json')),
    'bf16x3': (30, 'sad::halo256_kernel<',
               'sad::halo256_kernel (variant 30), split-bf16: patch-resident 256-channel x 16x16-pixel conv; the '
               'stride-1 layer3/4 convs (the last one fuses the average pool)',
               ('r06_pmc_traffic_bf16x3.json', 'r05_pmc_traffic_bf16x3.json')),
    'fp32': (13, 'sad::block_conv_kernel<float', 'sad::block_conv_kernel (variant 13), f32 MFMA', ()),
}


def traffic_file(dtype):
    return next((os.path.join(ROOT, 'profiles', f) for f in DOMINANT[dtype][3]
                 if os.path.exists(os.path.join(ROOT, 'profiles', f))), '')


FE_FLOP = 16.4e6               # per segment: window, rFFT 2.5 N log2 N x 251, |X|^2, mel, dB, stats
FE_BYTES = 256000 + 128512     # int16 PCM read + fp32 [128, 251] map written
HEADS = 6


def dominant_traffic(tr: dict, prefix: str = DOMINANT['bf16'][1]):
    """Memory-side bytes per launch (read + write) of the dominant kernel from a
    committed PMC traffic file (tools/profile_bench.sh): the launch-weighted mean
    over every record whose rocprof name starts with `prefix` (all template
    instantiations, e.g. the pooled and plain forms of variant 31).  None when no
    record matches or a matching record lacks its byte counts."""
    recs = [v for k, v in tr.items() if k.startswith(prefix)]
    if not recs or any(r.get('hbm_read_bytes') is None or r.get('hbm_write_bytes') is None for r in recs):
        return None
    w = [max(float(r.get('launches_per_step') or 1.0), 1e-9) for r in recs]
    tot = sum(wi * (r['hbm_read_bytes'] + r['hbm_write_bytes']) for wi, r in zip(w, recs))
    return round(tot / sum(w))


def cpu_model() -> str:
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or 'unknown'


def cpu_baseline(n_clips: int = 64, passes: int = 2):
    """configs[0]: the reference's CPU path (oracle restatement, fp32, torch CPU)
    on 64 synthetic 4 s / 32 kHz WAV clips and ONE sub-model, in the
    reference's structure: per-window front end (MelSpectrogram/AmplitudeToDB
    rebuilt per call, standardise, Resize, repeat(3)), windows batched by 128,
    the sub-model forward (inference_runner.py:144-174,276-289).  Timed twice:
    from decoded fp32 waveforms in memory, and from the WAV files (decode +
    mono + pad, preprocess_waveform :144-155, included)."""
    import tempfile

    import numpy as np
    from oracle import audio as oaudio
    from oracle import frontend as ofe
    from oracle import resnet as ores
    from sad import weights as sw
    from sad.audio import save_pcm16
    from sad.synth import synth_segment
    sd = sw.merged_state_dict(0, 1, False, bn_stats=sw.load_bn_stats(os.path.join(ROOT, 'tests', 'golden',
                                                                                    'bn_stats_n6.npz')))
    model = ores.load_merged_state(sd)
    cfg = ofe.SpectrogramConfig()
    pcm = [synth_segment(0, i) for i in range(n_clips)]

    def infer(waves):
        with torch.no_grad():
            for s in range(0, len(waves), 128):
                specs = torch.cat([ofe.waveform_to_spectrogram(w, 32000, cfg) for w in waves[s:s + 128]])
                model(specs)

    waves = [torch.from_numpy(p.astype(np.float32) / 32768.0) for p in pcm]
    infer(waves[:2])  # warm-up (allocator, thread pool)
    t0 = time.perf_counter()
    for _ in range(passes):
        infer(waves)
    t_mem = time.perf_counter() - t0
    with tempfile.TemporaryDirectory() as d:
        paths = []
        for i, p in enumerate(pcm):
            paths.append(os.path.join(d, f'clip{i:03d}.wav'))
            save_pcm16(paths[-1], p)
        t0 = time.perf_counter()
        for _ in range(passes):
            infer([oaudio.preprocess_waveform(p)[0] for p in paths])
        t_wav = time.perf_counter() - t0
    n = n_clips * passes
    return {'value': round(n / t_mem, 2), 'unit': 'segments/s', 'cores': torch.get_num_threads(), 'kind': 'port',
            'value_incl_wav_decode': round(n / t_wav, 2),
            'host': {'os_cpu_count': os.cpu_count(), 'torch_threads': torch.get_num_threads(),
                     'cpu_model': cpu_model(),
                     'threads_note': 'torch_threads = the CPU share one GPU gets on this box (the pool sets '
                                     'OMP_NUM_THREADS to 16 per GPU; os.cpu_count() counts the whole host, '
                                     'whose other cores belong to the other 7 GPUs); the reference runs '
                                     'inference single-process on the same share'},
            'sample': f'configs[0]: {n_clips} synthetic 4 s / 32 kHz clips x {passes} passes through the CPU '
                      f'oracle (per-window mel/dB/std/resize/repeat(3), windows batched by 128, 1 sub-model '
                      f'ResNet-18 + head, fp32): {t_mem:.1f} s from decoded waveforms; {t_wav:.1f} s from the WAV '
                      f'files (decode, mono, pad included)'}


def ingest_leg(eng, dev, minutes: float = 2.0, reps: int = 3):
    """SURVEY 8(f) row 1 on the device (sad.ingest, csrc/ingest.hip): one long
    44.1 kHz stereo int16 recording (synthesised in host memory, as a WAV's data
    chunk would be read) -> upload -> mono -> resample to 32 kHz -> silence test
    -> 4 s windows at main()'s overlap 0 read in place by the front end -> the
    headline engine.  Best of `reps`, HIP events per stage; the resample kernel
    priced against the fp32 VALU peak (2 K FLOP per output, K = 459 taps)."""
    import math

    import numpy as np
    from sad import engine, ingest
    sr = 44100
    T = int(minutes * 60 * sr)
    rs = np.random.RandomState(0)
    t = np.arange(T) / sr
    sig = 0.3 * np.sin(2 * np.pi * 440 * t) * (1 + 0.5 * np.sin(2 * np.pi * 0.1 * t)) + 0.05 * rs.randn(T)
    pcm = np.ascontiguousarray((np.stack([sig, np.roll(sig, 11)]).T * 20000).astype(np.int16)).reshape(-1)
    fe = engine.FrontEnd(dev)
    best = None
    for _ in range(reps + 1):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        ev[0].record()
        x = torch.from_numpy(pcm).to(dev)
        ev[1].record()
        wf = ingest.resampler(sr, 32000, dev)(ingest.mono(x, 2), 128000)
        ev[2].record()
        starts, _ = ingest.select_windows(wf, 32000, 4.0, 0.0, 1e-3)
        w = ingest.Windows(wf, starts, 128000)
        ev[3].record()
        eng.forward_maps(fe.windows(wf, w.offsets))
        ev[4].record()
        torch.cuda.synchronize()
        wall = time.perf_counter() - h0
        ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(4)]
        if best is None or wall < best[0]:
            best = (wall, ms, len(w), wf.shape[0])
    wall, ms, nwin, n_out = best
    K = 2 * math.ceil(6 * 441 / (320 * 0.99)) + 441
    flop = 2.0 * K * n_out
    return {'what': f'{minutes:g} min of 44.1 kHz stereo int16 -> device mono + torchaudio sinc resample + '
                    f'silence test + in-place windows (overlap 0) -> front end + ensemble',
            'windows': nwin, 'wall_ms': round(wall * 1e3, 3), 'segments_per_s': round(nwin / wall, 1),
            'h2d_ms': round(ms[0], 3), 'mono_resample_ms': round(ms[1], 3), 'select_ms': round(ms[2], 3),
            'frontend_ensemble_ms': round(ms[3], 3),
            'resample_roofline': {'bound': 'fp32 valu', 'taps': K, 'flop': flop,
                                  'achieved_tflops': round(flop / (ms[1] * 1e-3) / 1e12, 2),
                                  'peak_tflops': F32_PEAK_TFLOPS,
                                  'frac_lower_bound': round(flop / (ms[1] * 1e-3) / 1e12 / F32_PEAK_TFLOPS, 4),
                                  'note': 'timed with the mono kernel, so the fraction is a lower bound on the '
                                          'resample kernel alone'}}


class Mode:
    """One engine configuration timed on this rank's resident PCM: each step is
    front end -> backbone -> heads (-> all-gather).

    overlap: the next step's front end runs on a side stream while this step's
    backbone runs (two map slots; every step still takes its whole batch
    through every stage, the front end just starts one step early).  Round 5
    withdrew this after wrong logits in some pipelined steps; round 6 traced
    them to the front end's packed-FP32 instructions returning wrong values
    while MFMAs of the concurrent backbone ran on the same CUs, not to the
    hand-off; libsad is built without those instructions (DESIGN.md 5c,
    tests/test_gpu_handoff.py, tests/test_isa_scan.py).

    After the timed steps, ``run`` checks the LAST timed step's outputs: its
    merged logits must equal an untimed sequential forward of the same PCM bit
    for bit, and with N > 1 every rank's gathered logits must hold each rank's
    merged rows (``timed_output_check``; a mismatch raises)."""

    def __init__(self, sd, dev, dtype, micro_batch, B, world, overlap=False):
        from sad.engine import Engine
        self.eng = Engine(sd, dev, dtype=dtype, micro_batch=micro_batch)
        self.dtype, self.mb, self.B, self.world, self.dev = dtype, micro_batch, B, world, dev
        self.feats = torch.empty(B, 512, device=dev)
        self.logits = torch.empty(B, HEADS, 2, device=dev)
        self.merged = torch.empty(B, HEADS + 1, device=dev)
        self.gathered = torch.empty(world * B, HEADS + 1, device=dev) if world > 1 else None
        self.overlap = overlap
        if overlap:
            self.side = torch.cuda.Stream(dev)
            self.maps = [torch.empty(B, 128, 251, device=dev) for _ in range(2)]
            self.fe_done = [torch.cuda.Event(), torch.cuda.Event()]
            self.bb_done = [torch.cuda.Event(), torch.cuda.Event()]
            self.i = 0

    def _frontend_ahead(self, pcm, slot):
        # the slot's previous reader (the backbone two steps back) must be done
        self.side.wait_event(self.bb_done[slot])
        with torch.cuda.stream(self.side):
            self.eng.frontend(pcm, out=self.maps[slot])
        self.fe_done[slot].record(self.side)

    def step(self, pcm, ev=None):
        if ev is not None:
            ev[0].record()
        if self.overlap:  # this step's maps were computed during the previous step (the bench repeats one batch)
            slot = self.i & 1
            if self.i == 0:
                self._frontend_ahead(pcm, slot)
            cur = torch.cuda.current_stream()
            cur.wait_event(self.fe_done[slot])
            m = self.maps[slot]
        else:
            m = self.eng.frontend(pcm)
        if ev is not None:
            ev[1].record()
        self.eng.backbones[0](m, out=self.feats)
        if self.overlap:
            self.bb_done[slot].record(cur)
        if ev is not None:
            ev[2].record()
        self.eng.heads([self.feats], self.logits, self.merged)
        if ev is not None:
            ev[3].record()
        if self.gathered is not None:
            if dist.get_backend() == 'nccl':
                dist.all_gather_into_tensor(self.gathered, self.merged)
            else:  # gloo (the 2-rank one-GPU test)
                dist.all_gather(list(self.gathered.chunk(self.world)), self.merged)
        if ev is not None:
            ev[4].record()
        if self.overlap:  # the next step's front end, during this step's backbone
            self._frontend_ahead(pcm, slot ^ 1)
            self.i += 1

    def isolated(self, pcm, reps=5):
        """Front end and backbone timed alone (HIP events on the current
        stream, best of reps): the per-stage rooflines of an overlapped run,
        whose concurrent stages stretch each other."""
        cur = torch.cuda.current_stream()
        torch.cuda.synchronize()
        fe, bb = [], []
        for _ in range(reps):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record(cur)
            m = self.eng.frontend(pcm)
            e[1].record(cur)
            self.eng.backbones[0](m, out=self.feats)
            e[2].record(cur)
            torch.cuda.synchronize()
            fe.append(e[0].elapsed_time(e[1]))
            bb.append(e[1].elapsed_time(e[2]))
        return min(fe), min(bb)

    def run(self, pcm, steps, warmup, profile=True):
        from sad import _lib
        for _ in range(warmup):
            self.step(pcm)
        torch.cuda.synchronize()
        if self.world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(5)] for _ in range(steps)]
        t0 = time.perf_counter()
        for i in range(steps):
            if profile and i == steps - 1:
                # HIP events around each block-conv launch of the last timed step,
                # on its stream (events between launches cost ~5%, so one step only)
                _lib.call('sad_profile_begin')
            self.step(pcm, evs[i])
        torch.cuda.synchronize()
        if self.world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        k_ms, k_n, k_fl = _lib.ctypes.c_double(), _lib.I64(), _lib.ctypes.c_double()
        _lib.call('sad_profile_end', DOMINANT[self.dtype][0] if profile else -1, _lib.ctypes.byref(k_ms),
                  _lib.ctypes.byref(k_n), _lib.ctypes.byref(k_fl))
        mean = lambda a, b: sum(e[a].elapsed_time(e[b]) for e in evs) / steps  # noqa: E731
        r = {'elapsed': elapsed, 'fe_ms': mean(0, 1), 'bb_ms': mean(1, 2), 'heads_ms': mean(2, 3),
             'gather_ms': mean(3, 4), 'k_ms': k_ms.value, 'k_n': k_n.value, 'k_flop': k_fl.value}
        r['rank_ms_per_step'] = [round(elapsed * 1e3 / steps, 3)]
        r['rank_gather_ms'] = [round(r['gather_ms'], 4)]
        if self.world > 1:
            t = torch.tensor([elapsed, r['gather_ms']], device=self.dev, dtype=torch.float64)
            allt = [torch.empty_like(t) for _ in range(self.world)]
            dist.all_gather(allt, t)
            r['elapsed'] = max(x[0].item() for x in allt)
            r['rank_ms_per_step'] = [round(x[0].item() * 1e3 / steps, 3) for x in allt]
            r['rank_gather_ms'] = [round(x[1].item(), 4) for x in allt]
        r['ms'] = r['elapsed'] * 1e3 / steps
        r['value'] = self.world * self.B * steps / r['elapsed']
        r['timed_output_check'] = self.check_outputs(pcm)
        if self.overlap:
            # the stage rooflines from the stages run alone; the in-step events
            # bracket the wait for the side stream's front end, not its work
            r['fe_ms_in_step'], r['bb_ms_in_step'] = r['fe_ms'], r['bb_ms']
            r['fe_ms'], r['bb_ms'] = self.isolated(pcm)
        return r

    def check_outputs(self, pcm):
        """The last timed step's outputs against an untimed sequential forward
        (outside the timed region).  Raises on any difference."""
        last = self.merged.clone()
        _, ref = self.eng.forward_pcm(pcm)
        torch.cuda.synchronize()
        same = torch.equal(last, ref)
        chk = {'what': 'last timed step merged logits vs an untimed sequential forward of the same PCM, bit for bit',
               'bit_identical': same, 'max_abs_diff': (last - ref).abs().max().item()}
        if self.gathered is not None:
            rank = dist.get_rank()
            own = torch.equal(self.gathered.chunk(self.world)[rank], last)
            # every rank's gathered tensor must be the same bytes: compare a sum of its int32 words
            h = self.gathered.view(torch.int32).to(torch.int64).sum().reshape(1)
            hs = [torch.empty_like(h) for _ in range(self.world)]
            dist.all_gather(hs, h)
            ok = torch.tensor([int(own and same and len({int(x.item()) for x in hs}) == 1)], device=self.dev)
            oks = [torch.empty_like(ok) for _ in range(self.world)]
            dist.all_gather(oks, ok)
            chk['gathered_holds_own_rows'] = own
            chk['gathered_identical_on_all_ranks'] = len({int(x.item()) for x in hs}) == 1
            chk['all_ranks_ok'] = all(int(x.item()) == 1 for x in oks)
            same = chk['all_ranks_ok']
        if not same:
            raise RuntimeError(f'timed step outputs differ from the sequential forward: {chk}')
        return chk


def kernel_roofline(r, mfma_factor=1):
    """The dominant kernel's rate: algorithmic FLOPs / HIP-event time; the MFMA
    work it executes is mfma_factor x that (split-bf16: 3 products per MAC)."""
    n = max(r['k_n'], 1)
    alg = r['k_flop'] / (r['k_ms'] * 1e-3) / 1e12 if r['k_ms'] > 0 else 0.0
    return alg, alg * mfma_factor, {'launches': r['k_n'], 'launch_avg_us': round(r['k_ms'] * 1e3 / n, 2),
                                    'flop_per_launch': round(r['k_flop'] / n)}


def gemm_reference(dev, n=16384, reps=5):
    """hipBLASLt (torch.matmul) on a square bf16 GEMM, measured in this run on
    this GPU: what the vendor's best plain GEMM reaches here, next to the
    kernels' fractions of the 2.5 PFLOP/s spec (a reference point, not a peak)."""
    a = torch.randn(n, n, device=dev, dtype=torch.bfloat16)
    b = torch.randn(n, n, device=dev, dtype=torch.bfloat16)
    for _ in range(2):
        torch.matmul(a, b)
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        torch.matmul(a, b)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    tf = 2.0 * n ** 3 / (min(ts) * 1e-3) / 1e12
    del a, b
    return {'what': f'torch.matmul (hipBLASLt) bf16 {n}^3, random data, best of {reps}, measured in this run',
            'tflops': round(tf, 1), 'frac_of_peak': round(tf / BF16_PEAK_TFLOPS, 4)}


def decisions(merged):
    """Labels by the drop-in's interpret_multihead_logits (inference_runner.py:194-214)."""
    import inference_runner as ir
    names = [f'Synthetic{chr(65 + i)}' for i in range(HEADS)]
    return [ir.interpret_multihead_logits(row, 0.5, names)[0] for row in merged.cpu()]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=80)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--batch', type=int, default=2048, help='segments per GPU per step')
    ap.add_argument('--dtype', default='bf16', choices=['bf16', 'bf16x3', 'fp32'])
    ap.add_argument('--micro-batch', type=int, default=0,
                    help='segments per backbone launch sequence (0: 2048 bf16, 512 bf16x3, 128 fp32); stem/layer1 '
                         'run in sub-batches of SAD_FRONT_MB (256 for bf16 with the fused layer1, else 32), layers 2-4 on the whole micro-batch')
    ap.add_argument('--parity-steps', type=int, default=0, help='timed steps of the bf16x3 parity mode '
                                                                '(0: max(steps // 3, 3); -1: skip)')
    ap.add_argument('--fp32-steps', type=int, default=2, help='timed steps of the fp32 mode (N = 1; 0: skip)')
    ap.add_argument('--overlap-frontend', type=int, default=1,
                    help="1: each step's front end runs on a side stream during the previous step's backbone")
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--kernels-only', action='store_true',
                    help='profiling runs: only the headline mode (no parity/fp32 legs, accuracy or CPU baseline)')
    ap.add_argument('--backend', default='nccl', choices=['nccl', 'gloo'], help='gloo: tests only')
    ap.add_argument('--one-device', action='store_true', help='every rank on cuda:0 (2-rank test on one GPU)')
    args = ap.parse_args()

    if args.gpus > 1 and not launch.under_launcher():
        sys.exit(launch.relaunch(args.gpus, os.path.abspath(__file__), sys.argv[1:]))
    world, rank, local = launch.check_world(args.gpus)
    dev = torch.device('cuda', 0 if args.one_device else local)
    torch.cuda.set_device(dev)
    if world > 1:
        if args.backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
        else:
            dist.init_process_group('gloo')

    import numpy as np
    from sad import _lib
    from sad import weights as sw
    gold = os.path.join(ROOT, 'tests', 'golden')
    sd = sw.merged_state_dict(0, HEADS, False, bn_stats=sw.load_bn_stats(os.path.join(gold, 'bn_stats_n6.npz')))
    mbs = {'bf16': 2048, 'bf16x3': 512, 'fp32': 128}
    B = args.batch
    pcm = torch.empty(B, SEG, dtype=torch.int16, device=dev)
    _lib.call('sad_synth_pcm', 0, rank * B, B, SEG, _lib.ptr(pcm), _lib.stream_handle(dev))

    ov = bool(args.overlap_frontend)
    head = Mode(sd, dev, args.dtype, args.micro_batch or mbs[args.dtype], B, world, overlap=ov)
    r = head.run(pcm, args.steps, args.warmup)
    p_steps = max(args.steps // 3, 3) if args.parity_steps == 0 else args.parity_steps
    if args.kernels_only:
        p_steps, args.fp32_steps, args.no_cpu_baseline = -1, 0, True
    par_mode, par = None, None
    if p_steps > 0:
        if args.dtype == 'bf16x3':
            par_mode, par = head, r
        else:
            par_mode = Mode(sd, dev, 'bf16x3', mbs['bf16x3'], B, world, overlap=ov)
            par = par_mode.run(pcm, p_steps, 1)

    if rank == 0:
        from sad.engine import Engine
        # accuracy against the reference-generated fixtures (the bench model IS the golden n6 model) and
        # against the fp32 device path over this rank's whole batch
        fx = np.load(os.path.join(gold, 'golden_frontend.npz'))
        gm = np.load(os.path.join(gold, 'golden_models.npz'))['n6_merged']
        gpcm = torch.from_numpy(fx['pcm']).to(dev)
        if not args.kernels_only:
            e32 = Engine(sd, dev, dtype='fp32', micro_batch=mbs['fp32'])
            _, m32 = e32.forward_pcm(pcm)
            torch.cuda.synchronize()
            lab32 = decisions(m32)

        def accuracy(mode):
            if args.kernels_only:
                return None
            _, mg = mode.eng.forward_pcm(gpcm)
            torch.cuda.synchronize()
            lab = decisions(mode.merged)
            agree = sum(a == b for a, b in zip(lab, lab32)) / len(lab32)
            return {'max_dlogit_golden': round(float(np.abs(mg.cpu().numpy() - gm).max()), 7),
                    'golden_segments': int(gpcm.shape[0]),
                    'max_dlogit_vs_fp32_device': round((mode.merged - m32).abs().max().item(), 7),
                    'decision_agreement_vs_fp32_device': agree, 'segments_compared': B}

        peak = BF16_PEAK_TFLOPS if args.dtype != 'fp32' else F32_PEAK_TFLOPS
        fac = 3 if args.dtype == 'bf16x3' else 1
        alg, exe, kinfo = kernel_roofline(r, fac)
        def traffic_of(dtype):
            tf = traffic_file(dtype)
            if not tf:
                return None, None
            with open(tf) as f:
                return dominant_traffic(json.load(f), DOMINANT[dtype][1]), os.path.relpath(tf, ROOT)

        traffic, traffic_src = traffic_of(args.dtype)
        traffic_unit = ('memory-side bytes per launch = L2-miss traffic, Infinity-Cache hits included '
                        f'(FETCH_SIZE x2 + WRITE_SIZE, {traffic_src})')
        bb_alg = BACKBONE_FLOP * B / (r['bb_ms'] * 1e-3) / 1e12
        out = {
            'metric': '4s@32kHz segments/sec end-to-end (mel+ResNet+ensemble), 1/2/4/8 MI355X',
            'value': round(r['value'], 1), 'unit': 'segments/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(r['ms'], 3), 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': args.dtype,
            'data': 'synthetic int16 PCM (counter-hash PRNG, generated in HBM) + random-init ResNet-18/6 heads '
                    '(hash PRNG, BN-calibrated; = the golden n6 fixture model)',
            'config': {'workload': 'end-to-end inference: B int16 4 s segments resident in HBM -> mel front end '
                                   '-> ResNet-18@512x512 -> 6 binary heads -> merge (+RCCL all-gather of logits)',
                       'segments_per_gpu_per_step': B, 'heads': HEADS, 'distinct_backbones': 1,
                       'micro_batch': head.mb, 'parallelism': f'dp{world}',
                       'frontend_overlapped': ov,
                       'per_rank_ms_per_step': r['rank_ms_per_step'], 'per_rank_allgather_ms': r['rank_gather_ms']},
            'roofline': {'bound': 'mfma',
                         'kernel': DOMINANT[args.dtype][2],
                         'achieved': round(exe, 1), 'peak': peak, 'unit': 'TFLOP/s', 'frac': round(exe / peak, 4),
                         'traffic': traffic, 'traffic_unit': traffic_unit,
                         **kinfo,
                         'backbone': {'achieved': round(bb_alg * fac, 1), 'frac': round(bb_alg * fac / peak, 4),
                                      'ms_per_step': round(r['bb_ms'], 3), 'flop_per_segment': BACKBONE_FLOP,
                                      'what': 'fused resize+stem + 16 block-conv GEMMs + avgpool, HIP events '
                                              'around the backbone call in the timed steps'},
                         'gemm_reference': None if args.kernels_only or args.dtype == 'fp32' else gemm_reference(dev),
                         # front end (configs[1]): fused STFT/mel/dB + standardise, fp32 VALU-bound
                         # (16.4 MFLOP and 384,512 B per segment)
                         'frontend': {'ms_per_step': round(r['fe_ms'], 3),
                                      'achieved_tflops': round(FE_FLOP * B / (r['fe_ms'] * 1e-3) / 1e12, 2),
                                      'peak_tflops': F32_PEAK_TFLOPS,
                                      'frac': round(FE_FLOP * B / (r['fe_ms'] * 1e-3) / 1e12 / F32_PEAK_TFLOPS, 4),
                                      'achieved_gbps': round(FE_BYTES * B / (r['fe_ms'] * 1e-3) / 1e9, 1),
                                      'segments_per_s': round(B / (r['fe_ms'] * 1e-3), 1)}},
            'accuracy': accuracy(head),
            'timed_output_check': r['timed_output_check'],
            # HIP events on the main stream around each stage of the timed steps (means):
            # front-end wait (overlapped: the side stream's maps), backbone, heads + merge, all-gather
            'step_breakdown_ms': {'frontend_wait': round(r.get('fe_ms_in_step', r['fe_ms']), 3),
                                  'backbone': round(r.get('bb_ms_in_step', r['bb_ms']), 3),
                                  'heads_merge': round(r['heads_ms'], 3), 'allgather': round(r['gather_ms'], 4)},
        }
        if par is not None:
            palg, pexe, pinfo = kernel_roofline(par, 3)
            ptraffic, ptraffic_src = traffic_of('bf16x3')
            out['parity_mode'] = {
                'dtype': 'bf16x3', 'what': 'split-bf16: hi/lo bf16 operands, 3 bf16 MFMAs per product, fp32 '
                                           'accumulate (north-star parity mode)',
                'value': round(par['value'], 1), 'unit': 'segments/s', 'ms_per_step': round(par['ms'], 3),
                'steps': p_steps, 'micro_batch': par_mode.mb,
                'per_rank_ms_per_step': par['rank_ms_per_step'],
                'roofline': {'kernel': DOMINANT['bf16x3'][2], 'achieved': round(pexe, 1),
                             'unit': 'TFLOP/s (bf16 MFMA executed = 3 x algorithmic)', 'peak': BF16_PEAK_TFLOPS,
                             'frac': round(pexe / BF16_PEAK_TFLOPS, 4), 'algorithmic_tflops': round(palg, 1),
                             # a ratio, not a fraction: the f32-exact products run 3.x times faster than
                             # the f32 MFMA / VALU peak allows
                             'algorithmic_over_f32_peak_ratio': round(palg / F32_PEAK_TFLOPS, 4), **pinfo,
                             'traffic': ptraffic,
                             'traffic_unit': ('memory-side bytes per launch (FETCH_SIZE x2 + WRITE_SIZE, '
                                              f'{ptraffic_src})' if ptraffic_src else None),
                             'backbone_algorithmic_tflops': round(BACKBONE_FLOP * B / (par['bb_ms'] * 1e-3) / 1e12,
                                                                  1),
                             'backbone_executed_frac': round(3 * BACKBONE_FLOP * B / (par['bb_ms'] * 1e-3) / 1e12
                                                             / BF16_PEAK_TFLOPS, 4)},
                'accuracy': accuracy(par_mode) if par_mode is not head else out['accuracy'],
                'timed_output_check': par['timed_output_check']}
        if world == 1 and args.fp32_steps > 0 and args.dtype != 'fp32':
            f = Mode(sd, dev, 'fp32', mbs['fp32'], B, 1).run(pcm, args.fp32_steps, 1, profile=False)
            out['fp32_mode'] = {'value': round(f['value'], 1), 'unit': 'segments/s', 'ms_per_step': round(f['ms'], 3),
                                'steps': args.fp32_steps, 'peak': F32_PEAK_TFLOPS,
                                'backbone_tflops': round(BACKBONE_FLOP * B / (f['bb_ms'] * 1e-3) / 1e12, 1)}
        if world == 1 and not args.kernels_only:
            out['ingest'] = ingest_leg(head.eng, dev)
        if world == 1 and not args.no_cpu_baseline:
            out['cpu_baseline'] = cpu_baseline()
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
