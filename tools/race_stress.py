"""Determinism of each backbone kernel under memory contention: every kernel is
run once on a quiet device (reference), then REPS times while a side stream
runs the front end over a big batch and large device copies, and each output is
compared bit for bit with the reference.  A kernel whose LDS-DMA waits or
barriers leave a hazard that only timing hides shows up here as a mismatch."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'synthetic-audio-detection_amd')]
from sad import _lib  # noqa: E402
from sad import weights as sw  # noqa: E402
from sad.engine import Backbone, FrontEnd, block_conv, split_merged_state  # noqa: E402

DEV = torch.device('cuda:0')
REPS = int(os.environ.get('REPS', '12'))
g = torch.Generator(device=DEV).manual_seed(1)


def rnd(*shape, scale=1.0, relu=False):
    t = torch.randn(*shape, generator=g, device=DEV) * scale
    return (t.clamp_min(0) if relu else t).to(torch.bfloat16)


side = torch.cuda.Stream(DEV)
fe = FrontEnd(DEV)
noise_pcm = torch.randint(-20000, 20000, (1024, 128000), dtype=torch.int16, device=DEV, generator=g)
noise_map = torch.empty(1024, 128, 251, device=DEV)
big_a = torch.empty(512 * 1024 * 1024 // 4, device=DEV)
big_b = torch.empty_like(big_a)


def noise():
    with torch.cuda.stream(side):
        for _ in range(2):
            fe(noise_pcm, out=noise_map)
            big_b.copy_(big_a)


def conv_case(name, N, H, cin, cout, stride, sc=None, res=False, variant=0):
    x = rnd(N, H, H, cin, relu=True)
    Ho = H // stride
    K = 9 * cin + (cin if sc == 'ds' else 0)
    scx = rnd(N, 2 * H, 2 * H, cin // 2 if False else 64, relu=True) if sc == 'ds' else None
    if sc == 'ds':
        K = 9 * cin + 64
    w = rnd(cout, K, scale=(2.0 / K) ** 0.5)
    b = torch.randn(cout, generator=g, device=DEV) * 0.1
    r = rnd(N, Ho, Ho, cout, relu=True) if res else None
    kw = dict(sc=scx, sc_stride=2 if sc == 'ds' else 1, res=r, variant=variant)
    return name, lambda: block_conv(x, w, b, stride, 1, **kw)


def l1_case(N):
    x = rnd(N, 128, 128, 64, scale=0.7)
    w1 = rnd(64, 576, scale=(2.0 / 576) ** 0.5)
    w2 = torch.zeros(64, 640, dtype=torch.bfloat16, device=DEV)
    w2[:, :576] = rnd(64, 576, scale=(2.0 / 576) ** 0.5)
    w2[:, 576:] = torch.eye(64, dtype=torch.bfloat16, device=DEV)
    b1 = torch.randn(64, generator=g, device=DEV) * 0.1
    b2 = torch.randn(64, generator=g, device=DEV) * 0.1

    def run():
        out = torch.empty_like(x)
        _lib.call('sad_l1_block_run', _lib.ptr(x), N, 128, 128, _lib.ptr(w1), 576, _lib.ptr(b1), _lib.ptr(w2), 640,
                  _lib.ptr(b2), _lib.ptr(out), 0, _lib.stream_handle(DEV))
        return out
    return 'l1block v40', run


sd = sw.merged_state_dict(0, 6, False, bn_stats=sw.load_bn_stats(os.path.join(ROOT, 'tests', 'golden', 'bn_stats_n6.npz')))
_, bases, _ = split_merged_state(sd)
maps = fe(torch.randint(-20000, 20000, (96, 128000), dtype=torch.int16, device=DEV, generator=g))
bb = Backbone(bases[0], DEV, 'bf16', micro_batch=64)
cases = [
    ('backbone bf16 (96 seg, mb 64)', lambda: bb(maps)),
    ('stem', lambda: bb.stem(maps)),
    l1_case(64),
    conv_case('l2.0 conv1 v43', 64, 128, 64, 128, 2),
    conv_case('l2.0 conv2+ds v41', 64, 64, 128, 128, 1, sc='ds'),
    conv_case('l2.1 conv res v41', 64, 64, 128, 128, 1, res=True),
    conv_case('l2.1 conv v41', 64, 64, 128, 128, 1),
    conv_case('l3.0 conv1 v44', 128, 64, 128, 256, 2),
    conv_case('l4.0 conv1 v44', 128, 32, 256, 512, 2),
    conv_case('l3.0 conv1 v32', 128, 64, 128, 256, 2, variant=32),
    conv_case('l3 conv v31', 128, 32, 256, 256, 1),
]
torch.cuda.synchronize()
for name, fn in cases:
    ref = fn().clone()
    torch.cuda.synchronize()
    bad = 0
    for _ in range(REPS):
        noise()
        out = fn()
        torch.cuda.synchronize()
        if not torch.equal(out, ref):
            bad += 1
            d = (out.float() - ref.float()).abs()
            where = (d > 0).nonzero()
            print(f'  {name}: MISMATCH {int((d > 0).sum())} elements, max {d.max().item():.3g}, first at {where[0].tolist()}',
                  flush=True)
    print(f'{name}: {REPS - bad}/{REPS} bit-identical under contention', flush=True)
