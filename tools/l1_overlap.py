"""Layer1 conv (variant 25) launch overheads: per-image time vs launch size,
and whether two streams (kernel tails overlapping the next sub-chunk's ramp)
shorten a run of 32-segment launches.  Diagnostic, not a test."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'synthetic-audio-detection_amd'))
from sad.engine import block_conv  # noqa: E402

DEV = 'cuda:0'
torch.manual_seed(0)
w = (torch.randn(64, 576, device=DEV) * 0.06).to(torch.bfloat16)
b = torch.randn(64, device=DEV) * 0.1


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6


big = (torch.randn(512, 128, 128, 64, device=DEV)).to(torch.bfloat16)
for n in (32, 64, 128, 256, 512):
    x = big[:n]
    us = timeit(lambda: block_conv(x, w, b, 1, 1, k=3))
    usr = timeit(lambda: block_conv(x, w, b, 1, 1, res=x, k=3))
    print(f'N={n}: plain {us:.1f} us ({us / n:.3f}/img)  res {usr:.1f} us ({usr / n:.3f}/img)', flush=True)

subs = [big[i * 32:(i + 1) * 32] for i in range(16)]
s = [torch.cuda.current_stream(DEV), torch.cuda.Stream(DEV)]


def chains(nstream):
    # per sub-chunk: conv1 -> conv2 (+res) -> conv1 -> conv2 (+res), as layer1
    ev = torch.cuda.Event()
    ev.record(s[0])
    s[1].wait_event(ev)
    for i, x in enumerate(subs):
        with torch.cuda.stream(s[i % nstream]):
            t = block_conv(x, w, b, 1, 1, k=3)
            y = block_conv(t, w, b, 1, 1, res=x, k=3)
            t = block_conv(y, w, b, 1, 1, k=3)
            block_conv(t, w, b, 1, 1, res=y, k=3)
    ev2 = torch.cuda.Event()
    ev2.record(s[1])
    s[0].wait_event(ev2)


for rep in range(3):
    print(f'16 x 32-image layer1 chains: 1 stream {timeit(lambda: chains(1), 10):.0f} us, '
          f'2 streams {timeit(lambda: chains(2), 10):.0f} us', flush=True)
