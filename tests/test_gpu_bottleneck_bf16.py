"""GPU: one timm Bottleneck in bf16, conv by conv, on the kernels the resnet
plan picks (csrc/resnet.hip rn_chunk: variant 0 = default_block_variant), each
conv against its own arithmetic emulated on the CPU from the SAME bf16 inputs.

conv1 1x1 -> conv2 3x3/s -> conv3 1x1 + (identity residual in the epilogue,
variant 13 RES | the folded downsample as extra K columns).  conv2 runs on the
halo kernels (variant 25 at width 64, variant 20 at width 128) or the
implicit GEMM (stride 2).  Paths that only the bf16 Bottleneck nets use, so the
fp32 parity tests do not reach them.

Emulation: float64 conv + bias (+ shortcut / residual), ReLU, rounded once to
bf16.  The kernels accumulate in fp32 in another order, so an output may land
on the neighbouring bf16 value: the bar is 1 bf16 ulp (2^-7 relative) plus a
floor of 1e-3 of the tensor's rms for outputs near zero, against the 1e-1
relative pooled-feature bars of the end-to-end resnet50 test.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'


def _emu(x, w, bias, k, stride, sc=None, sc_stride=1, res=None):
    """x NHWC bf16, w [Cout, k*k*Cin (+Cin1)] bf16 -> NHWC bf16 (float64 math, one rounding)."""
    cin = x.shape[3]
    cout = w.shape[0]
    wt = w[:, :k * k * cin].double().reshape(cout, k, k, cin).permute(0, 3, 1, 2)
    y = F.conv2d(x.double().permute(0, 3, 1, 2), wt, stride=stride, padding=k // 2)
    if sc is not None:
        w1 = w[:, k * k * cin:].double()[:, :, None, None]
        y = y + F.conv2d(sc.double().permute(0, 3, 1, 2), w1, stride=sc_stride)
    y = y + bias.double()[None, :, None, None]
    if res is not None:
        y = y + res.double().permute(0, 3, 1, 2)
    return torch.relu(y).permute(0, 2, 3, 1).to(torch.bfloat16)


def _close(gpu, emu, what):
    g, e = gpu.cpu().double(), emu.double()
    bound = e.abs() * 2.0 ** -7 + 1e-3 * e.pow(2).mean().sqrt()
    d = (g - e).abs()
    assert bool((d <= bound).all()), f'{what}: max |d| {d.max().item():.3g}, worst excess {(d - bound).max().item():.3g}'
    return (d > 0).double().mean().item()


def _w(g, cout, K):
    return (torch.randn(cout, K, generator=g) * (2.0 / K) ** 0.5).to(torch.bfloat16)


# cin, width, stride, H, downsample
CASES = [(256, 64, 1, 32, False), (64, 64, 1, 32, True), (256, 128, 2, 32, True), (512, 128, 1, 16, False)]


@pytest.mark.parametrize('cin,width,stride,H,ds', CASES, ids=[f'c{c[0]}w{c[1]}s{c[2]}{"d" if c[4] else "i"}'
                                                            for c in CASES])
def test_bottleneck_bf16_convs_vs_emulation(cin, width, stride, H, ds):
    from sad.engine import block_conv
    g = torch.Generator().manual_seed(cin * 7 + width + stride)
    N, cout = 3, 4 * width
    if not ds:
        assert cin == cout
    x = torch.randn(N, H, H, cin, generator=g).to(torch.bfloat16)
    w1, w2 = _w(g, width, cin), _w(g, width, 9 * width)
    w3 = _w(g, cout, width + (cin if ds else 0))
    b1, b2, b3 = (torch.randn(c, generator=g) * 0.1 for c in (width, width, cout))
    xd = x.to(DEV)
    t1 = block_conv(xd, w1.to(DEV), b1.to(DEV), 1, 0, k=1)
    torch.cuda.synchronize()
    flips = [_close(t1, _emu(x, w1, b1, 1, 1), 'conv1 1x1')]
    t1h = t1.cpu()
    t2 = block_conv(t1, w2.to(DEV), b2.to(DEV), stride, 1, k=3)
    torch.cuda.synchronize()
    flips.append(_close(t2, _emu(t1h, w2, b2, 3, stride), f'conv2 3x3/{stride}'))
    t2h = t2.cpu()
    if ds:
        y = block_conv(t2, w3.to(DEV), b3.to(DEV), 1, 0, sc=xd, sc_stride=stride, k=1)
        ref = _emu(t2h, w3, b3, 1, 1, sc=x, sc_stride=stride)
    else:
        y = block_conv(t2, w3.to(DEV), b3.to(DEV), 1, 0, k=1, res=xd)
        ref = _emu(t2h, w3, b3, 1, 1, res=x)
    torch.cuda.synchronize()
    flips.append(_close(y, ref, 'conv3 1x1 + ' + ('downsample columns' if ds else 'residual')))
    print(f'share of outputs one bf16 ulp off the emulation: {flips}')
    assert max(flips) < 0.05
