"""GPU numerics of every block-conv tile variant (libsad block.hip / halo.hip)
against a plain torch fp32 conv of the same bf16-rounded operands.

One launch computes  act(conv3x3(x) [+ 1x1 shortcut(sc)] + bias [+ res])  -- the
BasicBlock halves of timm resnet18 (inference_runner.py:49-51).
The kernels accumulate in fp32 and round the output once to bf16, so the bar is
|out - ref| <= 1 bf16 ulp of |ref| (2^-8 relative) + a 1e-2 absolute floor for
summation-order noise near zero.  Variants of one kernel family sum K in the
same order, so their outputs must also agree bit for bit.

Shapes cover: several tiles per persistent workgroup, a ragged last pixel tile
(M % tile != 0), images smaller than one workgroup's pixel tile, the identity
shortcut as MFMA columns and as an epilogue residual, the strided downsample.
"""
import zlib

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'


def _ref(x, w, bias, stride, sc, sc_stride, res, relu, k=3):
    """fp32 NCHW reference of the block-conv contract on the bf16 operands."""
    cin = x.shape[3]
    wc = w[:, :k * k * cin].float().reshape(w.shape[0], k, k, cin).permute(0, 3, 1, 2)
    y = F.conv2d(x.float().permute(0, 3, 1, 2), wc, stride=stride, padding=k // 2)
    if sc is not None:
        w1 = w[:, k * k * cin:k * k * cin + sc.shape[3]].float()
        s = sc.float()[:, ::sc_stride, ::sc_stride, :]
        y = y + torch.einsum('nhwc,oc->nohw', s, w1)
    y = y + bias.view(1, -1, 1, 1)
    if res is not None:
        y = y + res.float().permute(0, 3, 1, 2)
    if relu:
        y = y.clamp_min(0)
    return y.permute(0, 2, 3, 1)


def _check(out, ref):
    d = (out.float() - ref).abs()
    bound = ref.abs() * 2.0 ** -8 + 1e-2
    assert bool((d <= bound).all()), f'max |d| {d.max().item():.3g}, worst excess {(d - bound).max().item():.3g}'


# name, N, H, Cin, Cout, stride, shortcut ('id' | 'ds' | 'res' | None), variants
CASES = [
    ('l1-res', 5, 128, 64, 64, 1, 'res', [20, 21, 25]),  # 320 tiles: 2 per workgroup on some
    ('l1-plain', 2, 48, 64, 64, 1, None, [9, 11, 16, 20, 25]),
    ('l1-res-32', 32, 128, 64, 64, 1, 'res', [25, 20]),   # the bench's sub-batch: 8 tiles per workgroup
    ('l2-res', 2, 32, 128, 128, 1, 'res', [20, 21, 22]),
    # a Bottleneck's conv2 (128 channels, no shortcut): halo family, GEMM family
    # (the two sum K in different orders, so they are not compared bitwise)
    ('l2-plain-halo', 3, 32, 128, 128, 1, None, [20, 21, 22]),
    ('l2-plain-halo-256', 2, 32, 128, 256, 1, None, [20, 22]),
    ('l2-plain-gemm', 3, 32, 128, 128, 1, None, [15, 10, 14, 19]),
    ('l2-s2', 3, 34, 64, 128, 2, None, [10, 12, 14, 15, 18, 19]),
    ('l2-ds', 2, 16, 128, 128, 1, 'ds', [10, 12, 14, 15, 18, 19]),
    ('l2-id', 3, 20, 128, 128, 1, 'id', [15, 19]),
    ('l3-id', 3, 14, 256, 256, 1, 'id', [13, 17, 10, 19]),
    ('l3-s2', 2, 18, 128, 256, 2, None, [13, 17, 19]),
    ('l4-ds', 5, 6, 512, 512, 1, 'ds', [13, 17, 19]),
    # variants 30 / 31 (patch-resident 256 x 256, halo256.hip / halo256r.hip):
    # chunk-outer K order, so their own cases; variant 31 starts its
    # accumulators at the bias (30 adds it after the sum), so the two are
    # compared with the reference only, not bitwise; ragged tile counts per
    # persistent workgroup (280 tiles on 256)
    ('l3-plain-30', 3, 32, 256, 256, 1, None, [30]),
    ('l3-plain-31', 3, 32, 256, 256, 1, None, [31]),
    ('l3-plain-30-ragged', 70, 32, 256, 256, 1, None, [30]),
    ('l3-plain-31-ragged', 70, 32, 256, 256, 1, None, [31]),
    ('l3-id-30', 2, 32, 256, 256, 1, 'id', [30]),
    ('l3-id-31', 2, 32, 256, 256, 1, 'id', [31]),
    ('l3-ds-30', 2, 16, 128, 256, 1, 'ds', [30]),
    ('l3-ds-31', 2, 16, 128, 256, 1, 'ds', [31]),
    ('l4-ds-30', 3, 16, 256, 512, 1, 'ds', [30]),
    ('l4-ds-31', 3, 16, 256, 512, 1, 'ds', [31]),
    ('l4-id-30', 5, 16, 512, 512, 1, 'id', [30]),
    ('l4-id-31', 5, 16, 512, 512, 1, 'id', [31]),
    ('l4-plain-30-rect', 2, 32, 512, 512, 1, None, [30]),
    ('l4-plain-31-rect', 2, 32, 512, 512, 1, None, [31]),
    # variant 31 with 128-channel tiles (layer2: 4 channel groups x 2 pixel
    # halves): plain, identity columns, the downsample from a 2x source (64 ch)
    ('l2-plain-31', 3, 64, 128, 128, 1, None, [31]),
    ('l2-plain-31-ragged', 9, 48, 128, 128, 1, None, [31]),
    ('l2-id-31', 2, 64, 128, 128, 1, 'id', [31]),
    ('l2-ds-31', 2, 32, 64, 128, 1, 'ds', [31]),
    ('l3-two-tiles-31', 2, 16, 128, 384, 1, None, [31]),
    # variant 41 (resident-weight 128 -> 128 conv, l2conv.hip): plain, with the
    # epilogue residual, fewer tiles than workgroups (45), more (320)
    ('l2-plain-41', 3, 64, 128, 128, 1, None, [41]),
    ('l2-res-41', 2, 64, 128, 128, 1, 'res', [41]),
    ('l2-res-41-ragged', 5, 48, 128, 128, 1, 'res', [41]),
    ('l2-res-41-many', 20, 64, 128, 128, 1, 'res', [41]),
    # variant 41's downsample form (layer2.0's conv2 + the 1x1/2 of the
    # 64-channel block input as two more K-steps)
    ('l2-ds-41', 2, 64, 64, 128, 1, 'ds', [41]),
    ('l2-ds-41-ragged', 5, 48, 64, 128, 1, 'ds', [41]),
    ('l2-ds-41-many', 20, 64, 64, 128, 1, 'ds', [41]),
    # variant 32 (patch-resident stride-2 3x3, halo256s2.hip): layer2/3/4's
    # first conv (128- and 256-channel tiles), few tiles (70 on 256
    # workgroups), many (600 on 256)
    ('l2-s2-32', 2, 128, 64, 128, 2, None, [32]),
    ('l3-s2-32', 3, 64, 128, 256, 2, None, [32]),
    ('l4-s2-32', 5, 32, 256, 512, 2, None, [32]),
    ('l3-s2-32-ragged', 70, 32, 128, 256, 2, None, [32]),
    ('l4-s2-32-many', 300, 32, 256, 512, 2, None, [32]),
    # variant 43 (resident-weight 64 -> 128 stride-2 conv, l2s2conv.hip):
    # layer2.0's conv1; one tile per image (both padded edges in one tile), fewer
    # tiles than workgroups, more (320 on 256: two per workgroup on some)
    ('l2-s2-43-one-tile', 3, 32, 64, 128, 2, None, [43]),
    ('l2-s2-43', 2, 128, 64, 128, 2, None, [43]),
    ('l2-s2-43-many', 20, 128, 64, 128, 2, None, [43]),
    # variant 44 (patch-resident stride-2 3x3 with 64-channel chunks in four
    # parity planes, halo256rs2.hip; round 5): layer3/4's conv1 (the default)
    # and layer2's (128-channel tiles: 4 channel groups x 2 pixel halves); one
    # tile per image, few tiles (70 on 256 workgroups), many (1,200 on 256)
    ('l3-s2-44', 3, 64, 128, 256, 2, None, [44]),
    ('l4-s2-44', 5, 32, 256, 512, 2, None, [44]),
    ('l3-s2-44-one-tile', 4, 32, 128, 256, 2, None, [44]),
    ('l3-s2-44-ragged', 70, 32, 128, 256, 2, None, [44]),
    ('l4-s2-44-many', 300, 32, 256, 512, 2, None, [44]),
    ('l2-s2-44', 2, 128, 64, 128, 2, None, [44]),
    ('l2-s2-44-many', 20, 64, 64, 128, 2, None, [44]),
    ('l3-s2-44-rect-c384', 2, 64, 192, 384, 2, None, [44]),
]


@pytest.mark.parametrize('name,N,H,Cin,Cout,stride,sc,variants', CASES, ids=[c[0] for c in CASES])
def test_block_conv_variants(name, N, H, Cin, Cout, stride, sc, variants):
    from sad.engine import block_conv
    g = torch.Generator().manual_seed(zlib.crc32(name.encode()))
    Ho = H // stride if stride == 2 else H
    cin0 = Cin
    scx = res = None
    cin1 = 0
    if sc == 'id':
        scx = torch.randn(N, Ho, Ho, Cout, generator=g).to(torch.bfloat16)
        cin1 = Cout
    elif sc == 'ds':
        scx = torch.randn(N, 2 * Ho, 2 * Ho, Cin, generator=g).to(torch.bfloat16)
        cin0, cin1 = Cout, Cin
        H = Ho
    elif sc == 'res':
        res = torch.randn(N, Ho, Ho, Cout, generator=g).to(torch.bfloat16)
    x = torch.randn(N, H, H, cin0, generator=g).to(torch.bfloat16)
    K = 9 * cin0 + cin1
    w = (torch.randn(Cout, K, generator=g) * (2.0 / K) ** 0.5).to(torch.bfloat16)
    bias = torch.randn(Cout, generator=g) * 0.1
    ref = _ref(x, w, bias, 1 if sc == 'ds' else stride, scx, 2 if sc == 'ds' else 1, res, True)
    xd, wd, bd = x.to(DEV), w.to(DEV), bias.to(DEV)
    scd = scx.to(DEV) if scx is not None else None
    rd = res.to(DEV) if res is not None else None
    first = None
    for v in variants:
        out = block_conv(xd, wd, bd, 1 if sc == 'ds' else stride, 1, sc=scd, sc_stride=2 if sc == 'ds' else 1,
                         relu=True, variant=v, res=rd)
        torch.cuda.synchronize()
        _check(out.cpu(), ref)
        if first is None:
            first = out
        else:
            assert torch.equal(out, first), f'variant {v} differs bitwise from variant {variants[0]}'


@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float32])
def test_bottleneck_1x1_epilogue_residual(dtype):
    """Variant 13 with RES: a Bottleneck's conv3 (1x1) + identity shortcut added
    in the epilogue (resnet.hip), ragged pixel tail (M = 588), and the same
    conv with the downsample as GEMM columns (K = width + cin)."""
    from sad.engine import block_conv
    g = torch.Generator().manual_seed(55)
    N, H, width, cout = 3, 14, 128, 512
    x = torch.randn(N, H, H, width, generator=g).to(torch.bfloat16)
    res = torch.randn(N, H, H, cout, generator=g).to(torch.bfloat16)
    w = (torch.randn(cout, width, generator=g) * (2.0 / width) ** 0.5).to(torch.bfloat16)
    bias = torch.randn(cout, generator=g) * 0.1
    ref = _ref(x, w, bias, 1, None, 1, res, True, k=1)
    out = block_conv(x.to(DEV, dtype), w.to(DEV, dtype), bias.to(DEV), 1, 0, relu=True, variant=13,
                     res=res.to(DEV, dtype), k=1)
    torch.cuda.synchronize()
    if dtype == torch.float32:
        assert (out.cpu() - ref).abs().max().item() <= 1e-4
    else:
        _check(out.cpu(), ref)
    # downsample folded as shortcut columns over a 2x larger source (stride 2)
    sc = torch.randn(N, 2 * H, 2 * H, 256, generator=g).to(torch.bfloat16)
    w2 = (torch.randn(cout, width + 256, generator=g) * (2.0 / (width + 256)) ** 0.5).to(torch.bfloat16)
    ref2 = _ref(x, w2, bias, 1, sc, 2, None, True, k=1)
    out2 = block_conv(x.to(DEV, dtype), w2.to(DEV, dtype), bias.to(DEV), 1, 0, sc=sc.to(DEV, dtype), sc_stride=2,
                      relu=True, k=1)
    torch.cuda.synchronize()
    if dtype == torch.float32:
        assert (out2.cpu() - ref2).abs().max().item() <= 1e-4
    else:
        _check(out2.cpu(), ref2)
