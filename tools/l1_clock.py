"""Shader clock and board power while the fused layer1 block (variant 40) runs
back to back with and without its memory operations (the kernel's timing
ablations: 1 = no next-tile patch DMA, 2 = no intermediate LDS stores, 4 = no
output stores).  Each configuration runs for --seconds while a thread samples
`rocm-smi --showclocks --showpower`; prints us per launch, median sclk and
power.  Question answered: is the ablations' gain (15-17 % each, far above the
instructions' issue cost, tools/mfma_ab.hip modes 14-21) a clock effect?"""
import argparse
import os
import re
import statistics
import subprocess
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'synthetic-audio-detection_amd'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'tests'))
import torch  # noqa: E402

from test_gpu_l1block import _fused, _operands  # noqa: E402


def sampler(stop, out):
    while not stop.is_set():
        try:
            r = subprocess.run(['rocm-smi', '--showclocks', '--showpower'], capture_output=True, text=True, timeout=20)
            s = re.search(r'sclk clock level: \S+ \((\d+)Mhz\)', r.stdout)
            p = re.search(r'Graphics Package Power \(W\): ([\d.]+)', r.stdout)
            if s and p:
                out.append((time.time(), int(s.group(1)), float(p.group(1))))
        except Exception:
            pass
        time.sleep(0.2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=256)
    ap.add_argument('--seconds', type=float, default=4.0)
    ap.add_argument('--ablate', type=int, nargs='+', default=[0, 1, 2, 4, 7, 0])
    args = ap.parse_args()
    ops = _operands(args.n, 128, 128, 1)
    for _ in range(3):
        _fused(*ops)
    torch.cuda.synchronize()
    for ab in args.ablate:
        samples = []
        stop = threading.Event()
        th = threading.Thread(target=sampler, args=(stop, samples), daemon=True)
        th.start()
        t0 = time.time()
        n = 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        while time.time() - t0 < args.seconds:
            for _ in range(50):
                _fused(*ops, ablate=ab)
            n += 50
            torch.cuda.synchronize()
        e1.record()
        torch.cuda.synchronize()
        stop.set()
        th.join()
        us = e0.elapsed_time(e1) * 1000.0 / n
        steady = [s for s in samples if s[0] - t0 > 1.0] or samples
        sclk = statistics.median(s[1] for s in steady) if steady else float('nan')
        pw = statistics.median(s[2] for s in steady) if steady else float('nan')
        print(f'ablate {ab}: {us:.1f} us per launch over {n} launches; sclk median {sclk:.0f} MHz, '
              f'power median {pw:.0f} W ({len(steady)} samples)', flush=True)
        time.sleep(1.0)


if __name__ == '__main__':
    main()
