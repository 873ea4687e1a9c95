"""GPU: the fused layer1 BasicBlock kernel (sad_l1_block_run, csrc/l1block.hip,
variant 40) against
  (1) the unfused path it replaces -- conv1, then conv2 + identity on the
      resident-weight halo kernel (variant 25), through sad_block_conv_run:
      both sum the taps in the same K order on the same MFMA, but the fused
      kernel starts its accumulators at the bias (conv2: bias + identity)
      where variant 25 adds them after the sum, so fp32 rounding differs and
      an intermediate value can land one bf16 ulp apart; bar as (2), and at
      most 1 % of the outputs may differ at all;
  (2) a torch fp32 reference of timm's BasicBlock with BN folded
      (inference_runner.py:49-51): mid = bf16(relu(conv(x, w1) + b1)),
      out = relu(conv(mid, w2) + b2 + x); bar: 1 bf16 ulp of |ref| + 1e-2.
Shapes: one 16 x 16 image (every tile edge is an image border), non-square
maps, fewer tiles than workgroups, more tiles than workgroups (ragged
per-workgroup tile ranges), and the engine's 32-image sub-batch.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'


def _operands(N, H, W, seed):
    g = torch.Generator().manual_seed(seed)
    x = (torch.randn(N, H, W, 64, generator=g) * 0.7).clamp_min(-0.5).to(torch.bfloat16)
    w1 = (torch.randn(64, 576, generator=g) * (2.0 / 576) ** 0.5).to(torch.bfloat16)
    w2 = torch.zeros(64, 640, dtype=torch.bfloat16)  # the engine's layout: 64 identity K columns after the taps
    w2[:, :576] = (torch.randn(64, 576, generator=g) * (2.0 / 576) ** 0.5).to(torch.bfloat16)
    w2[:, 576:] = torch.eye(64, dtype=torch.bfloat16)
    b1 = torch.randn(64, generator=g) * 0.1
    b2 = torch.randn(64, generator=g) * 0.1
    return [t.to(DEV) for t in (x, w1, b1, w2, b2)]


def _fused(x, w1, b1, w2, b2, ablate=0):
    from sad import _lib
    N, H, W, _ = x.shape
    out = torch.empty_like(x)
    _lib.call('sad_l1_block_run', _lib.ptr(x), N, H, W, _lib.ptr(w1), 576, _lib.ptr(b1), _lib.ptr(w2), 640,
              _lib.ptr(b2), _lib.ptr(out), ablate, _lib.stream_handle(torch.device(DEV)))
    return out


def _unfused(x, w1, b1, w2, b2):
    from sad import _lib
    N, H, W, _ = x.shape
    s = _lib.stream_handle(torch.device(DEV))
    mid = torch.empty_like(x)
    out = torch.empty_like(x)
    _lib.call('sad_block_conv_run', _lib.ptr(x), N, H, W, 64, None, 0, 0, 0, 1, _lib.ptr(w1), 576, _lib.ptr(b1),
              None, _lib.ptr(mid), 64, 3, 1, 1, 1, _lib.SAD_BF16, 25, s)
    _lib.call('sad_block_conv_run', _lib.ptr(mid), N, H, W, 64, None, 0, 0, 0, 1, _lib.ptr(w2), 640, _lib.ptr(b2),
              _lib.ptr(x), _lib.ptr(out), 64, 3, 1, 1, 1, _lib.SAD_BF16, 25, s)
    return out


def _torch_ref(x, w1, b1, w2, b2):
    xf = x.float().permute(0, 3, 1, 2)
    k1 = w1.float().reshape(64, 3, 3, 64).permute(0, 3, 1, 2)
    k2 = w2[:, :576].float().reshape(64, 3, 3, 64).permute(0, 3, 1, 2)
    mid = F.conv2d(xf, k1, padding=1).add(b1.view(1, -1, 1, 1)).clamp_min(0).to(torch.bfloat16).float()
    y = F.conv2d(mid, k2, padding=1).add(b2.view(1, -1, 1, 1)).add(xf).clamp_min(0)
    return y.permute(0, 2, 3, 1)


# (round 4: tiles run down column strips and a tile that continues one copies
# its top halo from the tile above; 37 x 128^2, 40 x 64 x 48 and 300 x 48 x 16
# give workgroups several tiles with ranges that start and end mid-strip)
@pytest.mark.parametrize('N,H,W', [(1, 16, 16), (2, 48, 32), (3, 128, 128), (5, 64, 80), (37, 128, 128),
                                   (40, 64, 48), (300, 48, 16)])
def test_fused_block_matches_unfused(N, H, W):
    ops = _operands(N, H, W, N * 1000 + H + W)
    out = _fused(*ops)
    ref = _unfused(*ops)
    torch.cuda.synchronize()
    assert torch.isfinite(out.float()).all()
    d = (out.float() - ref.float()).abs()
    bound = ref.float().abs() * 2.0 ** -8 + 1e-2
    assert bool((d <= bound).all()), f'max |d| {d.max().item():.3g}'
    nd = (out != ref).sum().item()
    assert nd <= out.numel() // 100, f'{nd} of {out.numel()} outputs differ'


@pytest.mark.parametrize('N,H,W', [(1, 16, 16), (2, 48, 32), (32, 128, 128)])
def test_fused_block_vs_torch_fp32(N, H, W):
    ops = _operands(N, H, W, 7 + N + H)
    out = _fused(*ops).float()
    ref = _torch_ref(*ops)
    d = (out - ref).abs()
    bound = ref.abs() * 2.0 ** -8 + 1e-2
    assert bool((d <= bound).all()), f'max |d| {d.max().item():.3g}'


def test_fused_block_rejects_bad_shapes():
    from sad import _lib
    x, w1, b1, w2, b2 = _operands(1, 16, 16, 3)
    out = torch.empty_like(x)
    with pytest.raises(RuntimeError, match='multiples of 16'):
        _lib.call('sad_l1_block_run', _lib.ptr(x), 1, 16, 8, _lib.ptr(w1), 576, _lib.ptr(b1), _lib.ptr(w2), 640,
                  _lib.ptr(b2), _lib.ptr(out), 0, _lib.stream_handle(torch.device(DEV)))
    with pytest.raises(RuntimeError, match='overlap'):
        _lib.call('sad_l1_block_run', _lib.ptr(x), 1, 16, 16, _lib.ptr(w1), 576, _lib.ptr(b1), _lib.ptr(w2), 640,
                  _lib.ptr(b2), _lib.ptr(x), 0, _lib.stream_handle(torch.device(DEV)))
