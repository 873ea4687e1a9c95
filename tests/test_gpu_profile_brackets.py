"""GPU: the kernel-timing brackets behind bench.py's roofline (sad_profile_begin
/ sad_profile_end, include/sad.h) count KERNEL launches.  At 2,048 segments
layer3.0's conv2 + downsample passes the 2 GiB buffer range and runs as two
image-range launches inside one bracket, so variant 31 shows 7 launches per
backbone pass (5 stride-1 layer3/4 convs, one split in two, plus the pooled
last conv), and the bracket's FLOPs are the algorithmic FLOPs of those convs."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_profile_counts_kernel_launches():
    sys.path.insert(0, ROOT)
    import bench
    from sad import _lib
    from sad import weights as sw
    from sad.engine import Engine
    dev = torch.device('cuda:0')
    sd = sw.merged_state_dict(0, bench.HEADS, False,
                              bn_stats=sw.load_bn_stats(os.path.join(ROOT, 'tests', 'golden', 'bn_stats_n6.npz')))
    B = 2048
    eng = Engine(sd, dev, dtype='bf16', micro_batch=B)
    pcm = torch.empty(B, bench.SEG, dtype=torch.int16, device=dev)
    _lib.call('sad_synth_pcm', 5, 0, B, bench.SEG, _lib.ptr(pcm), _lib.stream_handle(dev))
    m = eng.frontend(pcm)
    feats = torch.empty(B, 512, device=dev)
    eng.backbones[0](m, out=feats)
    torch.cuda.synchronize()
    _lib.call('sad_profile_begin')
    eng.backbones[0](m, out=feats)
    ms, n, fl = _lib.ctypes.c_double(), _lib.I64(), _lib.ctypes.c_double()
    _lib.call('sad_profile_end', 31, _lib.ctypes.byref(ms), _lib.ctypes.byref(n), _lib.ctypes.byref(fl))
    assert n.value == 7
    assert ms.value > 0
    # layer3: 3 convs 256 -> 256 at 32x32 (+ the 1x1/2 downsample of 128 channels
    # on the first), layer4: 2 stride-1 convs at 16x16 (+ 1x1/2 of 256 channels
    # on the first; the pooled last conv is one of them): 2*M*Cout*K each
    l3 = 2.0 * B * 32 * 32 * 256 * (3 * 9 * 256 + 128)
    l4 = 2.0 * B * 16 * 16 * 512 * (3 * 9 * 512 + 256)
    assert abs(fl.value - (l3 + l4)) / (l3 + l4) < 1e-9
    assert torch.isfinite(feats).all()
