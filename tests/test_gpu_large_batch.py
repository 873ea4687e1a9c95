"""GPU: operands past the kernels' 2 GiB buffer-offset range.

launch_block_conv runs such a batch as consecutive launches over image ranges;
every conv is independent per image, so the result must equal, bit for bit,
the same conv run image range by image range -- and the whole backbone at a
micro-batch whose layer2 input is 2.1 GiB (1,024 segments in bf16) must equal
the micro-batch-512 run.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'


def _rand(shape, seed, scale=1.0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return (torch.randn(shape, generator=g, device=DEV) * scale).to(torch.bfloat16)


@pytest.mark.parametrize('case', ['l1_res_halo', 'l2_s2_gemm', 'l3_ds_gemm'])
def test_split_launch_equals_image_ranges(case):
    from sad.engine import block_conv
    if case == 'l1_res_halo':        # variant 25 + residual: in0 and res 2.3 GB each
        N, H, cin, cout, stride, k = 1100, 128, 64, 64, 1, 3
    elif case == 'l2_s2_gemm':       # layer2.0.conv1 (stride 2) on the GEMM kernels: in0 2.3 GB
        N, H, cin, cout, stride, k = 1100, 128, 64, 128, 2, 3
    else:                            # layer3.0.conv2 + downsample columns: in1 (shortcut source) 2.3 GB
        N, H, cin, cout, stride, k = 2200, 32, 256, 256, 1, 3
    x = _rand((N, H, H, cin), 1)
    sc = res = None
    K = k * k * cin
    if case == 'l1_res_halo':
        res = _rand((N, H, H, cout), 2)
    if case == 'l3_ds_gemm':
        sc = _rand((N, 2 * H, 2 * H, 128), 3)
        K += 128
    w = _rand((cout, K), 4, (2.0 / K) ** 0.5)
    b = torch.randn(cout, device=DEV) * 0.1
    kw = dict(sc=sc, sc_stride=2 if sc is not None else 1, res=res, k=k)
    big = block_conv(x, w, b, stride, 1, **kw)
    half = N // 2
    parts = []
    for lo, hi in ((0, half), (half, N)):
        kp = dict(kw)
        if sc is not None:
            kp['sc'] = sc[lo:hi]
        if res is not None:
            kp['res'] = res[lo:hi]
        parts.append(block_conv(x[lo:hi], w, b, stride, 1, **kp))
    torch.cuda.synchronize()
    assert torch.equal(big, torch.cat(parts))
    assert big.float().abs().sum() > 0


def test_backbone_micro_batch_1024_equals_512():
    import os

    from conftest import GOLDEN
    from sad import _lib, weights as sw
    from sad.engine import Engine
    sd = sw.merged_state_dict(0, 6, False, bn_stats=sw.load_bn_stats(os.path.join(GOLDEN, 'bn_stats_n6.npz')))
    B = 1024
    pcm = torch.empty(B, 128000, dtype=torch.int16, device=DEV)
    _lib.call('sad_synth_pcm', 7, 0, B, 128000, _lib.ptr(pcm), _lib.stream_handle(torch.device(DEV)))
    _, m1024 = Engine(sd, DEV, dtype='bf16', micro_batch=1024).forward_pcm(pcm)
    _, m512 = Engine(sd, DEV, dtype='bf16', micro_batch=512).forward_pcm(pcm)
    torch.cuda.synchronize()
    assert torch.equal(m1024, m512)


def test_backbone_micro_batch_2048_equals_1024():
    """The bench's micro-batch (2,048 segments: layer1's output is 4 GiB, so
    every layer2 conv runs as image-range launches) against two 1,024-segment
    micro-batches, bit for bit."""
    import os

    from conftest import GOLDEN
    from sad import _lib, weights as sw
    from sad.engine import Engine
    sd = sw.merged_state_dict(0, 6, False, bn_stats=sw.load_bn_stats(os.path.join(GOLDEN, 'bn_stats_n6.npz')))
    B = 2048
    pcm = torch.empty(B, 128000, dtype=torch.int16, device=DEV)
    _lib.call('sad_synth_pcm', 11, 0, B, 128000, _lib.ptr(pcm), _lib.stream_handle(torch.device(DEV)))
    _, m2048 = Engine(sd, DEV, dtype='bf16', micro_batch=2048).forward_pcm(pcm)
    _, m1024 = Engine(sd, DEV, dtype='bf16', micro_batch=1024).forward_pcm(pcm)
    torch.cuda.synchronize()
    assert torch.equal(m2048, m1024)


def test_backbone_x3_micro_batch_512_equals_256():
    """The parity mode at the bench's micro-batch (512 segments in split bf16:
    layer1's output is 512 x 128^2 x 128 x 2 B = 2^31 B, past the 32-bit buffer
    range, so layer2.0's convs run as split-bf16 image-range launches) against
    two 256-segment micro-batches, bit for bit."""
    import os

    from conftest import GOLDEN
    from sad import _lib, weights as sw
    from sad.engine import Engine
    sd = sw.merged_state_dict(0, 6, False, bn_stats=sw.load_bn_stats(os.path.join(GOLDEN, 'bn_stats_n6.npz')))
    B = 512
    pcm = torch.empty(B, 128000, dtype=torch.int16, device=DEV)
    _lib.call('sad_synth_pcm', 13, 0, B, 128000, _lib.ptr(pcm), _lib.stream_handle(torch.device(DEV)))
    _, m512 = Engine(sd, DEV, dtype='bf16x3', micro_batch=512).forward_pcm(pcm)
    _, m256 = Engine(sd, DEV, dtype='bf16x3', micro_batch=256).forward_pcm(pcm)
    torch.cuda.synchronize()
    assert torch.isfinite(m512).all()
    assert torch.equal(m512, m256)
