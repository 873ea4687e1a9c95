"""GPU: the bf16 training stem in one pass (sad_stem_train_run: conv.hip
stem_bf16_kernel<false, true> + batch-statistic finalize + bn1/ReLU on the
sign(gamma)-max-pooled raw conv) against float64 torch on the same bf16 image
and the same bf16 (pack mode 4) weights, with some bn1 gammas negative (the
min-pool side of the sign trick) and one zero.

Tolerances: batch mean / var and the running stats relative 1e-5 of the
channel's scale; output |d| <= 2^-8 (|scale| |m'| + |ref|) + 1e-5, i.e. the
bf16 rounding of the pooled raw map and of the output.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'


def test_stem_train_vs_float64():
    from sad import _lib
    g = torch.Generator().manual_seed(11)
    n = 3
    img = (torch.randn(n, 512, 512, generator=g) * 0.7).bfloat16()
    w = torch.randn(64, 3, 7, 7, generator=g) * 0.05
    gamma = torch.rand(64, generator=g) + 0.5
    gamma[::5] *= -1.0
    gamma[7] = 0.0
    beta = torch.randn(64, generator=g) * 0.1
    rm0, rv0 = torch.randn(64, generator=g) * 0.1, torch.rand(64, generator=g) + 0.5
    s = _lib.stream_handle(torch.device(DEV))
    wd = w.to(DEV)
    wp = torch.empty(64 * 64, dtype=torch.bfloat16, device=DEV)
    _lib.call('sad_pack_conv_weight_run', _lib.ptr(wd), 64, 3, 7, 4, _lib.SAD_BF16, _lib.ptr(wp), s)
    w8 = wp.view(64, 8, 8).cpu().double()
    assert torch.all(w8[:, 7, :] == 0) and torch.all(w8[:, :, 7] == 0)
    wk = w8[:, :7, :7].unsqueeze(1)                            # [64, 1, 7, 7], the bf16 weights used
    y = F.conv2d(img.double().unsqueeze(1), wk, stride=2, padding=3)  # [n, 64, 256, 256]
    mean = y.mean(dim=(0, 2, 3))
    var = y.var(dim=(0, 2, 3), unbiased=False)
    istd = 1.0 / torch.sqrt(var + 1e-5)
    scale = gamma.double() * istd
    shift = beta.double() - mean * scale
    ref = F.max_pool2d(torch.relu(y * scale.view(1, -1, 1, 1) + shift.view(1, -1, 1, 1)), 3, 2, 1)
    mp = F.max_pool2d(y * torch.where(gamma < 0, -1.0, 1.0).double().view(1, -1, 1, 1), 3, 2, 1)

    sz = _lib.SZ()
    _lib.call('sad_stem_train_workspace_size', n, _lib.ctypes.byref(sz))
    ws = torch.empty(sz.value, dtype=torch.uint8, device=DEV)
    out = torch.empty(n, 128, 128, 64, dtype=torch.bfloat16, device=DEV)
    st = torch.empty(256, device=DEV)
    rm, rv = rm0.clone().to(DEV), rv0.clone().to(DEV)
    imgd, gd, bd = img.to(DEV), gamma.to(DEV), beta.to(DEV)
    _lib.call('sad_stem_train_run', _lib.ptr(imgd), n, _lib.ptr(wp), _lib.ptr(gd), _lib.ptr(bd), 1e-5, 0.1,
              _lib.ptr(rm), _lib.ptr(rv), _lib.ptr(st), _lib.ptr(out), _lib.ptr(ws), ws.numel(), s)
    torch.cuda.synchronize()
    st = st.cpu().double()
    sd = torch.sqrt(var)
    assert ((st[:64] - mean).abs() / sd).max() <= 1e-5
    assert ((st[64:128] - istd).abs() / istd).max() <= 1e-5
    P = n * 256 * 256
    assert ((rm.cpu().double() - (0.9 * rm0.double() + 0.1 * mean)).abs() / sd).max() <= 1e-5
    rv_ref = 0.9 * rv0.double() + 0.1 * var * P / (P - 1)
    assert ((rv.cpu().double() - rv_ref).abs() / rv_ref).max() <= 1e-5
    got = out.cpu().double().permute(0, 3, 1, 2)
    bound = 2.0 ** -8 * (scale.abs().view(1, -1, 1, 1) * mp.abs() + ref.abs()) + 1e-5
    d = (got - ref).abs()
    print(f'stem train: max |d| {d.max().item():.3e}, max |d|/bound {(d / bound).max().item():.3f}')
    assert torch.all(d <= bound)
