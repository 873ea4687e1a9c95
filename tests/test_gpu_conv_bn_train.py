"""GPU: train-mode conv + BatchNorm statistics (sad_conv_bn_train_run).  bf16
sums the statistics in the conv epilogues of the block-conv variants 13 / 15
and the halo kernels 20 / 25 (csrc/block.hip, csrc/halo.hip, StatAcc), fp32
runs the conv and the bn_reduce pass.  Reference: float64 torch conv on the same
bf16 (or fp32) inputs and weights, batch mean / biased var, running stats
(momentum 0.1, unbiased var).

Tolerances: mean |d| <= 1e-5 * std, invstd and running var relative 1e-5
(fp32 accumulation of the sums; the unfused bf16 path sums the bf16-rounded
output: 2e-3); raw output relative 1e-2 (bf16 storage) or 1e-5 (fp32).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'


@pytest.mark.parametrize('dtype,N,H,cin,cout,k,stride,pad,fused', [
    ('bf16', 4, 64, 64, 64, 3, 1, 1, 1),       # layer1: halo variant 25
    ('bf16', 4, 32, 128, 128, 3, 1, 1, 1),     # layer2 stride 1: resident-weight variant 41 (round 4; 16 tiles)
    ('bf16', 64, 64, 128, 128, 3, 1, 1, 1),    # ... at the trainer's 64 segments: 1,024 tiles on 256 workgroups
    ('bf16', 64, 64, 64, 128, 3, 2, 1, 1),     # layer2.0 conv1 at 64 segments: variant 43 (round 4; one tile per workgroup)
    ('bf16', 64, 128, 64, 128, 3, 2, 1, 1),    # ... 1,024 tiles on 256 workgroups
    ('bf16', 64, 64, 64, 128, 1, 2, 0, 1),     # layer2.0 downsample: variant 15
    ('bf16', 64, 32, 256, 256, 3, 1, 1, 1),    # layer3 at 64 segments: variant 13
    ('bf16', 64, 16, 512, 512, 3, 1, 1, 1),    # layer4 at 64 segments: 128 tiles of 256x256 -> variant 15
    ('bf16', 509, 16, 256, 512, 1, 2, 0, 1),   # variant 13 with a ragged last pixel tile (M = 32576)
    ('bf16', 4, 16, 256, 256, 3, 1, 1, 1),     # tiny map: variant 15
    ('bf16', 4, 32, 64, 64, 3, 2, 1, 0),       # Cout 64, stride 2: variant 9, conv + bn_reduce
    ('fp32', 2, 16, 256, 256, 3, 1, 1, 0),     # fp32: conv + bn_reduce
    # a Bottleneck layer1 conv3 (1x1, 64 -> 256 at 128^2) at 260 images: the
    # 2.18 GB output passes the 32-bit buffer range, so the conv runs as
    # image-range launches and the statistics take the unfused bn_reduce path
    ('bf16', 260, 128, 64, 256, 1, 1, 0, 0),
])
def test_conv_bn_train_vs_float64(dtype, N, H, cin, cout, k, stride, pad, fused):
    from sad import _lib
    code = _lib.SAD_BF16 if dtype == 'bf16' else _lib.SAD_F32
    tdt = torch.bfloat16 if dtype == 'bf16' else torch.float32
    g = torch.Generator().manual_seed(N + H + cin + cout + k)
    x = torch.randn(N, H, H, cin, generator=g).clamp_min(0).to(tdt)
    w = torch.randn(cout, cin, k, k, generator=g) * (2.0 / (k * k * cin)) ** 0.5
    gamma = torch.rand(cout, generator=g) + 0.5
    beta = torch.randn(cout, generator=g) * 0.1
    rm0, rv0 = torch.randn(cout, generator=g).double() * 0.1, torch.rand(cout, generator=g).double() + 0.5
    s = _lib.stream_handle(torch.device(DEV))
    wd = w.to(DEV)
    wp = torch.empty(w.numel(), dtype=tdt, device=DEV)
    _lib.call('sad_pack_conv_weight_run', _lib.ptr(wd), cout, cin, k, 0, code, _lib.ptr(wp), s)
    wq = wp.view(cout, k, k, cin).permute(0, 3, 1, 2).double()       # the weights the kernel used
    y = F.conv2d(x.to(DEV).double().permute(0, 3, 1, 2), wq, stride=stride, padding=pad)  # float64 on the device
    mean = y.mean(dim=(0, 2, 3))
    var = y.var(dim=(0, 2, 3), unbiased=False)
    P = y.numel() // cout

    Ho = y.shape[2]
    sz = _lib.SZ()
    _lib.call('sad_conv_bn_train_workspace_size', N, H, H, cout, k, stride, pad, _lib.ctypes.byref(sz))
    ws = torch.empty(sz.value // 4 + 1, device=DEV)
    out = torch.empty(N, Ho, Ho, cout, dtype=tdt, device=DEV)
    st = torch.empty(4 * cout, device=DEV)
    rm, rv = rm0.float().to(DEV), rv0.float().to(DEV)
    mean, var = mean.cpu(), var.cpu()
    fz = _lib.ctypes.c_int32(-1)
    xd, gd, bd = x.to(DEV), gamma.to(DEV), beta.to(DEV)
    _lib.call('sad_conv_bn_train_run', _lib.ptr(xd), N, H, H, cin, _lib.ptr(wp), cout, k, stride, pad, code,
              _lib.ptr(gd), _lib.ptr(bd), 1e-5, 0.1, _lib.ptr(rm), _lib.ptr(rv), _lib.ptr(st), _lib.ptr(out),
              _lib.ptr(ws), ws.numel() * 4, _lib.ctypes.byref(fz), s)
    torch.cuda.synchronize()
    assert fz.value == fused
    st = st.cpu().double()
    sd = var.sqrt()
    e_mean = ((st[:cout] - mean).abs() / sd).max().item()
    istd = 1.0 / torch.sqrt(var + 1e-5)
    e_istd = ((st[cout:2 * cout] - istd).abs() / istd).max().item()
    e_rm = ((rm.cpu().double() - (0.9 * rm0.double() + 0.1 * mean)).abs() / sd).max().item()
    rv_ref = 0.9 * rv0.double() + 0.1 * var * P / (P - 1)
    e_rv = ((rv.cpu().double() - rv_ref).abs() / rv_ref).max().item()
    ref_out = y.permute(0, 2, 3, 1)
    e_out = ((out.double() - ref_out).abs().max() / ref_out.abs().max()).item()
    print(f'{dtype} {cin}->{cout} k{k} s{stride} H{H}: fused {fz.value} mean {e_mean:.1e} istd {e_istd:.1e} '
          f'rm {e_rm:.1e} rv {e_rv:.1e} out {e_out:.1e}')
    # unfused bf16 sums the stored (bf16-rounded) output: 2^-9 relative per value
    tol = 1e-5 if fused or dtype == 'fp32' else 2e-3
    assert max(e_mean, e_istd, e_rm, e_rv) <= tol
    assert e_out <= (1e-2 if dtype == 'bf16' else 1e-5)
    # scale / shift as bn_apply consumes them
    sc = gamma.double() * istd
    assert ((st[2 * cout:3 * cout] - sc).abs() / sc.abs()).max() <= tol
