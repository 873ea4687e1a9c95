"""GPU: the trainer's hand-written MFMA contractions over the pixel axis
(csrc/wgrad.hip) -- conv weight gradient (every stride / kernel size the
ResNet-18/34 backward uses, split-K partials, beta accumulate) and the strided
conv input gradient (dcol GEMM + col2im) -- against float64 torch autograd of
the same conv on the same (bf16-representable) values.

Tolerance: max |d| <= 1e-5 * max |ref| (fp32 accumulation; bf16 operands are
exact in both).  Shapes: layer4 / layer3 training shapes, a ragged one
(channels not a multiple of the 128-wide tile, odd map size) and an empty batch.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'


def _dt(dtype):
    from sad import _lib
    return (_lib.SAD_BF16, torch.bfloat16) if dtype == 'bf16' else (_lib.SAD_F32, torch.float32)


def _wgrad_ref(x, dy, k, stride, pad):
    xd = x.double().permute(0, 3, 1, 2).requires_grad_(False)
    w = torch.zeros(dy.shape[-1], x.shape[-1], k, k, dtype=torch.float64, requires_grad=True)
    y = F.conv2d(xd, w, stride=stride, padding=pad)
    y.backward(dy.double().permute(0, 3, 1, 2))
    return w.grad


@pytest.mark.parametrize('dtype', ['bf16', 'fp32'])
@pytest.mark.parametrize('N,H,cin,cout,k,stride,pad', [
    (4, 16, 512, 512, 3, 1, 1),    # layer4 conv2
    (4, 32, 256, 512, 3, 2, 1),    # layer4.0 conv1
    (4, 32, 256, 512, 1, 2, 0),    # layer4.0 downsample
    (2, 32, 256, 256, 3, 1, 1),    # layer3 conv
    (3, 9, 24, 40, 3, 2, 1),       # ragged
])
def test_wgrad_vs_float64(dtype, N, H, cin, cout, k, stride, pad):
    from sad import _lib
    code, tdt = _dt(dtype)
    g = torch.Generator().manual_seed(N * 131 + H + cin + k + stride)
    Ho = (H + 2 * pad - k) // stride + 1
    x = torch.randn(N, H, H, cin, generator=g).clamp_min(0).to(tdt)
    dy = (torch.randn(N, Ho, Ho, cout, generator=g) * 0.1).to(tdt)
    ref = _wgrad_ref(x, dy, k, stride, pad)
    prev = torch.randn(cout, cin, k, k, generator=g)
    for beta in (0.0, 1.0):
        dw = prev.clone().to(DEV)
        sz = _lib.SZ()
        _lib.call('sad_conv_wgrad_workspace_size', N, H, H, cin, cout, k, stride, pad, code, _lib.ctypes.byref(sz))
        ws = torch.empty(max(sz.value, 1), dtype=torch.uint8, device=DEV)
        xd, dyd = x.to(DEV), dy.to(DEV)
        _lib.call('sad_conv_wgrad_run', _lib.ptr(xd), N, H, H, cin, _lib.ptr(dyd), cout, k, stride, pad, code, beta,
                  _lib.ptr(dw), _lib.ptr(ws), ws.numel(), _lib.stream_handle(torch.device(DEV)))
        torch.cuda.synchronize()
        want = ref + beta * prev.double()
        err = ((dw.cpu().double() - want).abs().max() / want.abs().max()).item()
        print(f'wgrad {dtype} N{N} H{H} {cin}->{cout} k{k} s{stride} beta {beta}: rel err {err:.2e} '
              f'(ws {sz.value / 2**20:.1f} MiB)')
        assert err <= 1e-5, err


def test_wgrad_empty_batch_scales_by_beta():
    from sad import _lib
    dw = torch.ones(8, 8, 3, 3, device=DEV)
    x = torch.zeros(16, device=DEV)  # never read: N = 0
    _lib.call('sad_conv_wgrad_run', _lib.ptr(x), 0, 4, 4, 8, _lib.ptr(x), 8, 3, 1, 1, _lib.SAD_F32, 0.5,
              _lib.ptr(dw), None, 0, _lib.stream_handle(torch.device(DEV)))
    torch.cuda.synchronize()
    assert torch.equal(dw.cpu(), torch.full((8, 8, 3, 3), 0.5))


@pytest.mark.parametrize('dtype', ['bf16', 'fp32'])
@pytest.mark.parametrize('N,H,cin,cout,k,stride,pad', [
    (4, 32, 256, 512, 3, 2, 1),    # layer4.0 conv1 (into layer3 when it trains)
    (4, 32, 256, 512, 1, 2, 0),    # layer4.0 downsample
    (2, 64, 128, 256, 3, 2, 1),    # layer3.0 conv1
    (8, 9, 24, 40, 3, 2, 1),       # ragged (P = 200, J = 216)
])
def test_strided_dgrad_vs_float64(dtype, N, H, cin, cout, k, stride, pad):
    from sad import _lib
    code, tdt = _dt(dtype)
    g = torch.Generator().manual_seed(N * 7 + H + cin + k)
    Ho = (H + 2 * pad - k) // stride + 1
    w = torch.randn(cout, cin, k, k, generator=g) * (2.0 / (k * k * cin)) ** 0.5
    wq = w.to(tdt)
    dy = (torch.randn(N, Ho, Ho, cout, generator=g) * 0.1).to(tdt)
    x = torch.zeros(N, cin, H, H, dtype=torch.float64, requires_grad=True)
    F.conv2d(x, wq.double(), stride=stride, padding=pad).backward(dy.double().permute(0, 3, 1, 2))
    ref = x.grad.permute(0, 2, 3, 1)
    prev = torch.randn(N, H, H, cin, generator=g).to(tdt)
    wp = torch.empty(w.numel(), dtype=tdt, device=DEV)
    wd = w.to(DEV)
    s = _lib.stream_handle(torch.device(DEV))
    _lib.call('sad_pack_conv_weight_run', _lib.ptr(wd), cout, cin, k, 3, code, _lib.ptr(wp), s)
    sz = _lib.SZ()
    _lib.call('sad_conv_dgrad_workspace_size', N, Ho, Ho, cout, cin, k, code, _lib.ctypes.byref(sz))
    ws = torch.empty(sz.value, dtype=torch.uint8, device=DEV)
    dyd = dy.to(DEV)
    for acc in (0, 1):
        dx = prev.clone().to(DEV)
        _lib.call('sad_conv_dgrad_run', _lib.ptr(dyd), N, Ho, Ho, cout, _lib.ptr(wp), cin, H, H, k, stride, pad, code,
                  acc, _lib.ptr(dx), _lib.ptr(ws), ws.numel(), s)
        torch.cuda.synchronize()
        want = ref + (prev.double() if acc else 0)
        got = dx.cpu().double()
        err = ((got - want).abs().max() / want.abs().max()).item()
        print(f'dgrad {dtype} N{N} H{H} {cin}<-{cout} k{k} s{stride} acc {acc}: rel err {err:.2e}')
        # the result is stored in the compute dtype: bf16 rounds it (2^-9 relative)
        assert err <= (4e-3 if dtype == 'bf16' else 1e-5), err


@pytest.mark.parametrize('N,H,cin,cout,k,stride,pad', [
    (64, 16, 512, 512, 3, 1, 1),   # bench_train.py's layer4 conv2 (P = 16384)
    (64, 32, 256, 512, 3, 2, 1),
    (64, 32, 256, 512, 1, 2, 0),
])
def test_wgrad_bench_shapes_bf16(N, H, cin, cout, k, stride, pad):
    """The 64-segment shapes of bench_train.py, reference float64 on the device."""
    from sad import _lib
    g = torch.Generator(device=DEV).manual_seed(5)
    Ho = (H + 2 * pad - k) // stride + 1
    x = torch.randn(N, H, H, cin, generator=g, device=DEV).clamp_min(0).bfloat16()
    dy = (torch.randn(N, Ho, Ho, cout, generator=g, device=DEV) * 0.01).bfloat16()
    ref = torch.nn.grad.conv2d_weight(x.double().permute(0, 3, 1, 2), (cout, cin, k, k),
                                      dy.double().permute(0, 3, 1, 2), stride=stride, padding=pad)
    dw = torch.empty(cout, cin, k, k, device=DEV)
    sz = _lib.SZ()
    _lib.call('sad_conv_wgrad_workspace_size', N, H, H, cin, cout, k, stride, pad, _lib.SAD_BF16,
              _lib.ctypes.byref(sz))
    ws = torch.empty(sz.value, dtype=torch.uint8, device=DEV)
    _lib.call('sad_conv_wgrad_run', _lib.ptr(x), N, H, H, cin, _lib.ptr(dy), cout, k, stride, pad, _lib.SAD_BF16,
              0.0, _lib.ptr(dw), _lib.ptr(ws), ws.numel(), _lib.stream_handle(torch.device(DEV)))
    torch.cuda.synchronize()
    err = ((dw.double() - ref).abs().max() / ref.abs().max()).item()
    print(f'wgrad bench shape N{N} H{H} {cin}->{cout} k{k} s{stride}: rel err {err:.2e}')
    assert err <= 1e-5, err
