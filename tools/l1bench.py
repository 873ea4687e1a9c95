"""Time the fused layer1 BasicBlock (variant 40) against the two unfused
launches it replaces (variant 25 conv1 + conv2/residual), on N-image batches
of 128 x 128 x 64 bf16 maps.  10 back-to-back launches x 3 (median), after
warm-up; reports us per block and TFLOP/s of the block's algorithmic work
(2 convs x 2 * N*128*128*64*576)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'synthetic-audio-detection_amd'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'tests'))
import torch  # noqa: E402

from test_gpu_l1block import _fused, _operands, _unfused  # noqa: E402


def timeit(fn, iters=10, reps=3):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1000.0 / iters)
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, nargs='+', default=[32, 256])
    ap.add_argument('--ablate', type=int, nargs='*', default=[])
    args = ap.parse_args()
    for n in args.n:
        ops = _operands(n, 128, 128, 1)
        fl = 2 * 2.0 * n * 128 * 128 * 64 * 576
        tf = timeit(lambda: _fused(*ops))
        tu = timeit(lambda: _unfused(*ops))
        print(f'N={n}: fused {tf:.1f} us ({fl / tf / 1e6:.0f} TFLOP/s), unfused v25 {tu:.1f} us '
              f'({fl / tu / 1e6:.0f} TFLOP/s), speedup {tu / tf:.3f}', flush=True)
        for ab in args.ablate:
            ta = timeit(lambda: _fused(*ops, ablate=ab))
            print(f'  ablate {ab}: {ta:.1f} us', flush=True)


if __name__ == '__main__':
    main()
