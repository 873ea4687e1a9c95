"""GPU parity of the split-bf16 parity mode (dtype 'bf16x3', SAD_BF16X3).

Every activation and weight is stored as hi = bf16(v), lo = bf16(v - hi) and
each product runs as W_hi.X_hi + W_lo.X_hi + W_hi.X_lo on the bf16 MFMA with
fp32 accumulation (csrc/block.hip, csrc/conv.hip stem_bf16_kernel<true>).
Operands carry ~2^-17 relative error, so the mode meets the north-star bar
|dlogit| <= 1e-3 against the fp32 reference (CPU emulation: 8.4e-5 on the
golden n6 model) at 3x the bf16 MFMA work instead of 16x (f32 MFMA).

Tolerances:
  * one block-conv launch vs float64 torch conv: relative 1e-4 of the output scale
  * stem / pooled features vs the fp32 oracle: relative 1e-4 / 2e-4
  * logits vs the reference-generated fixtures: |d| <= 1e-3 (north star)
  * logits vs the fp32 device path over a 512-segment batch: |d| <= 1e-3
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import merged_sd

pytestmark = pytest.mark.gpu

DEV = 'cuda:0'


def _conv_ref(x, w, stride, pad, sc=None, wsc=None, sc_stride=1, bias=None, relu=True):
    """float64 NHWC reference: conv(x) [+ 1x1/sc_stride(sc)] + bias, ReLU."""
    y = F.conv2d(x.permute(0, 3, 1, 2).double(), w.double(), None, stride=stride, padding=pad)
    if sc is not None:
        y = y + F.conv2d(sc.permute(0, 3, 1, 2).double(), wsc.double()[:, :, None, None], None, stride=sc_stride)
    if bias is not None:
        y = y + bias.double().view(1, -1, 1, 1)
    if relu:
        y = y.clamp_min(0)
    return y.permute(0, 2, 3, 1)


@pytest.mark.parametrize('cin,cout,H,stride,shortcut,variant', [
    (64, 64, 32, 1, 'identity', 0),     # layer1 shape class: variant 9
    (64, 128, 32, 2, 'downsample', 0),  # layer2.0 conv2 + downsample: variant 15
    (128, 256, 16, 1, None, 0),         # variant 13 (256x256 rolling prefetch)
    (256, 256, 16, 1, 'identity', 13),
    (256, 256, 16, 1, 'identity', 30),  # patch-resident 256 x 256 (halo256.hip)
    (128, 256, 32, 2, 'downsample', 30),
    (256, 512, 32, 1, None, 30),
    (128, 128, 16, 1, None, 10),
    # variant 31's split form (halo256r.hip, round 4): the layer3/4 stride-1 default
    (256, 256, 16, 1, 'identity', 31),
    (256, 256, 32, 1, 'identity', 31),
    (128, 256, 32, 2, 'downsample', 31),
    (256, 512, 32, 1, None, 31),
    (512, 512, 16, 1, 'identity', 31),
    # ... and its 128-channel tiles (layer2's stride-1 convs in the parity mode)
    (128, 128, 16, 1, 'identity', 31),
    (64, 128, 32, 2, 'downsample', 31),
    (128, 128, 48, 1, None, 31),
    # variant 44's split form (round 5): every stride-2 conv1 of the parity mode
    (128, 256, 64, 2, None, 44),        # layer3.0 conv1
    (256, 512, 32, 2, None, 44),        # layer4.0 conv1 (two channel tiles)
    (64, 128, 128, 2, None, 44),        # layer2.0 conv1 (128-channel tiles)
    (128, 256, 32, 2, None, 44),        # one tile per image
])
def test_block_conv_x3_vs_float64(cin, cout, H, stride, shortcut, variant):
    from sad.engine import block_conv, from_split, to_split
    g = torch.Generator().manual_seed(cin * 7 + cout + H)
    N = 3
    x = torch.randn(N, H, H, cin, generator=g).clamp_min(0)  # post-ReLU activations
    w = torch.randn(cout, cin, 3, 3, generator=g) * (2.0 / (9 * cin)) ** 0.5
    bias = torch.randn(cout, generator=g) * 0.1
    Ho = H // stride
    wk = w.permute(0, 2, 3, 1).reshape(cout, 9 * cin)
    sc = wsc = None
    if shortcut == 'identity':
        assert cin == cout and stride == 1
        xin = x
        x = torch.randn(N, H, H, cin, generator=g).clamp_min(0)  # conv input; shortcut = xin
        sc, wsc, ss = xin, torch.eye(cout), 1
    elif shortcut == 'downsample':
        # conv2 of a downsample block: 3x3/s1 over a [Ho,Ho,cout] map + 1x1/2 over x
        xin = x
        x = torch.randn(N, Ho, Ho, cout, generator=g).clamp_min(0)
        w = torch.randn(cout, cout, 3, 3, generator=g) * (2.0 / (9 * cout)) ** 0.5
        wk = w.permute(0, 2, 3, 1).reshape(cout, 9 * cout)
        sc, wsc, ss = xin, torch.randn(cout, cin, generator=g) * (1.0 / cin) ** 0.5, 2
        stride = 1
    wfull = torch.cat([wk, wsc], 1) if sc is not None else wk
    ref = _conv_ref(x, w, stride, 1, sc, wsc, ss if sc is not None else 1, bias)
    out = block_conv(to_split(x).to(DEV), to_split(wfull).to(DEV), bias.to(DEV), stride=stride, pad=1,
                     sc=to_split(sc).to(DEV) if sc is not None else None, sc_stride=ss if sc is not None else 1,
                     variant=variant, split=True)
    torch.cuda.synchronize()
    got = from_split(out.cpu()).double()
    err = ((got - ref).abs().max() / ref.abs().max()).item()
    print(f'x3 block conv {cin}->{cout} H{H} s{stride} {shortcut} v{variant}: rel err {err:.3e}')
    assert err <= 1e-4, err


def _parts(t):
    hi = t.to(torch.bfloat16).float()
    return hi, (t - hi).to(torch.bfloat16).float()


@pytest.mark.parametrize('cin,cout,H,k,stride,shortcut,variant', [
    (64, 64, 32, 1, 1, None, 9),          # a Bottleneck conv1 (1x1, width 64)
    (64, 64, 32, 3, 1, None, 9),          # its 3x3 conv2
    (128, 128, 32, 3, 2, None, 15),       # layer2.0 conv2 (3x3/s2, width 128)
    (128, 256, 16, 1, 1, 'res', 13),      # conv3 + identity as the epilogue residual
    (64, 256, 32, 1, 1, 'downsample', 13),  # conv3 + the 1x1 downsample as K columns
    (256, 512, 16, 1, 1, None, 15),       # small grid: variant 15
])
def test_block_conv_four_products(cin, cout, H, k, stride, shortcut, variant):
    """The four-product split-bf16 form (SAD_CONV_FOUR_PRODUCTS: + W_lo.X_lo,
    the deep Bottleneck plans' convs, resnet.hip) against float64 convs of the
    same split operands, next to the three-product form on the same variant:
    each is closer (RMS over the output) to its own arithmetic's reference than
    to the other's, and the four-product result is within 1e-4 of the output
    scale of the exact conv of the stored operands."""
    from sad.engine import block_conv, from_split, to_split
    g = torch.Generator().manual_seed(cin + 3 * cout + H + k)
    N = 3
    x = torch.randn(N, H, H, cin, generator=g).clamp_min(0)
    w = torch.randn(cout, cin, k, k, generator=g) * (2.0 / (k * k * cin)) ** 0.5
    bias = torch.randn(cout, generator=g) * 0.1
    Ho = (H + 2 * (k // 2) - k) // stride + 1
    wk = w.permute(0, 2, 3, 1).reshape(cout, k * k * cin)
    sc = wsc = res = None
    if shortcut == 'downsample':
        sc = torch.randn(N, 2 * Ho, 2 * Ho, 2 * cin, generator=g).clamp_min(0)
        wsc = torch.randn(cout, 2 * cin, generator=g) * (1.0 / (2 * cin)) ** 0.5
    elif shortcut == 'res':
        res = torch.randn(N, Ho, Ho, cout, generator=g).clamp_min(0)
    wfull = torch.cat([wk, wsc], 1) if sc is not None else wk
    xs, ws = from_split(to_split(x)), from_split(to_split(wfull))  # the stored operand values
    scs = from_split(to_split(sc)) if sc is not None else None
    rs = from_split(to_split(res)).double() if res is not None else 0
    w4 = ws[:, :k * k * cin].reshape(cout, k, k, cin).permute(0, 3, 1, 2)
    wsc4 = ws[:, k * k * cin:] if sc is not None else None

    def pre(xv, wv, scv, wscv):  # conv [+ shortcut] in float64, no bias / ReLU
        return _conv_ref(xv, wv, stride, k // 2, scv, wscv, 2, None, relu=False)

    full = pre(xs, w4, scs, wsc4)
    xl, wl = _parts(xs)[1], _parts(w4)[1]
    lolo = pre(xl, wl, _parts(scs)[1] if sc is not None else None, _parts(wsc4)[1] if sc is not None else None)
    post = lambda y: (y + bias.double().view(1, 1, 1, -1) + rs).clamp_min(0)  # noqa: E731
    ref4, ref3 = post(full), post(full - lolo)
    outs = {}
    for four in (False, True):
        out = block_conv(to_split(x).to(DEV), to_split(wfull).to(DEV), bias.to(DEV), stride=stride, pad=k // 2,
                         sc=to_split(sc).to(DEV) if sc is not None else None, sc_stride=2,
                         res=to_split(res).to(DEV) if res is not None else None, variant=variant, k=k,
                         split=True, four=four)
        torch.cuda.synchronize()
        outs[four] = from_split(out.cpu()).double()
    rms = lambda a, b: ((a - b) ** 2).mean().sqrt().item()  # noqa: E731
    d4, d4x = rms(outs[True], ref4), rms(outs[True], ref3)
    d3, d3x = rms(outs[False], ref3), rms(outs[False], ref4)
    err = ((outs[True] - ref4).abs().max() / ref4.abs().max()).item()
    print(f'four products {cin}->{cout} k{k} s{stride} {shortcut} v{variant}: rms vs 4-ref {d4:.3e} '
          f'(vs 3-ref {d4x:.3e}); three products rms vs 3-ref {d3:.3e} (vs 4-ref {d3x:.3e}); max rel {err:.3e}')
    assert d4 < d4x and d3 < d3x
    assert err <= 1e-4, err


@pytest.mark.parametrize('c,H,res,variant', [(64, 32, True, 20), (64, 48, False, 20), (128, 16, True, 20),
                                             (128, 32, False, 20), (64, 32, True, 26), (64, 48, False, 26),
                                             (64, 16, True, 26), (64, 80, True, 26),
                                             # variant 42 (round 4): the parity mode's layer1 default
                                             (64, 32, True, 42), (64, 48, False, 42), (64, 16, True, 42),
                                             (64, 80, True, 42), (64, 160, True, 42), (64, 160, False, 42)])
def test_halo_conv_x3_vs_float64(c, H, res, variant):
    """The split-bf16 halo kernels (variant 20: weight ring, layer2 stride-1
    convs; variant 26: resident weights, half the channels per workgroup,
    layer1; variant 42: register-resident weights, all channels per workgroup,
    layer1) with the identity shortcut as an epilogue residual, vs float64
    (H = 160: 300 tiles, more than workgroups)."""
    from sad.engine import block_conv, from_split, to_split
    g = torch.Generator().manual_seed(c + H + int(res))
    N = 3
    x = torch.randn(N, H, H, c, generator=g).clamp_min(0)
    r = torch.randn(N, H, H, c, generator=g).clamp_min(0) if res else None
    w = torch.randn(c, c, 3, 3, generator=g) * (2.0 / (9 * c)) ** 0.5
    bias = torch.randn(c, generator=g) * 0.1
    y = F.conv2d(x.permute(0, 3, 1, 2).double(), w.double(), bias.double(), padding=1).permute(0, 2, 3, 1)
    ref = (y + (r.double() if res else 0)).clamp_min(0)
    wk = w.permute(0, 2, 3, 1).reshape(c, 9 * c)
    out = block_conv(to_split(x).to(DEV), to_split(wk).to(DEV), bias.to(DEV), variant=variant, split=True,
                     res=to_split(r).to(DEV) if res else None)
    torch.cuda.synchronize()
    err = ((from_split(out.cpu()).double() - ref).abs().max() / ref.abs().max()).item()
    print(f'x3 halo conv v{variant} c{c} H{H} res={res}: rel err {err:.3e}')
    assert err <= 1e-4, err


def test_stem_x3_vs_oracle(golden_frontend):
    from oracle import frontend as ofe
    from oracle import resnet as ores
    from sad.engine import Backbone, split_merged_state
    sd = merged_sd('n6')
    _, bases, _ = split_merged_state(sd)
    bb = Backbone(bases[0], DEV, 'bf16x3')
    maps = torch.from_numpy(golden_frontend['std_map'])
    out = bb.stem(maps.to(DEV)).cpu()
    base = ores.load_merged_state(sd).sub_models[0].base
    with torch.no_grad():
        img = ofe.resize_bilinear(maps.unsqueeze(1), (512, 512)).repeat(1, 3, 1, 1)
        ref = base.maxpool(base.act1(base.bn1(base.conv1(img)))).permute(0, 2, 3, 1)
    err = ((out - ref).abs().max() / ref.abs().max()).item()
    print(f'stem bf16x3 rel err {err:.3e}')
    assert err <= 1e-4


def test_backbone_x3_vs_oracle(golden_frontend, golden_models):
    from sad.engine import Backbone, split_merged_state
    _, bases, _ = split_merged_state(merged_sd('n6'))
    bb = Backbone(bases[0], DEV, 'bf16x3')
    maps = torch.from_numpy(golden_frontend['std_map']).to(DEV)
    feats, l4 = bb.debug(maps)
    fused = bb(maps)
    torch.cuda.synchronize()
    ref = torch.from_numpy(golden_models['n6_feats0'])
    err = ((feats.cpu() - ref).abs().max() / ref.abs().max()).item()
    errf = ((fused.cpu() - ref).abs().max() / ref.abs().max()).item()
    print(f'backbone bf16x3 pooled rel err {err:.3e} (fused pool {errf:.3e})')
    assert err <= 2e-4 and errf <= 2e-4
    assert torch.allclose(feats, l4.mean(dim=(1, 2)), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize('tag', ['n6', 'n2'])
def test_logits_x3_match_reference(golden_frontend, golden_models, tag):
    """North-star gate for the parity mode: int16 PCM -> merged logits."""
    from sad.engine import Engine
    eng = Engine(merged_sd(tag), DEV, dtype='bf16x3', micro_batch=3)  # ragged: 4 = 3 + 1
    pcm = torch.from_numpy(golden_frontend['pcm']).to(DEV)
    logits, merged = eng.forward_pcm(pcm)
    torch.cuda.synchronize()
    d_merged = np.abs(merged.cpu().numpy() - golden_models[f'{tag}_merged']).max()
    d_heads = np.abs(logits.cpu().numpy() - golden_models[f'{tag}_per_head']).max()
    print(f'{tag} bf16x3 max|dlogit| merged {d_merged:.3e} per-head {d_heads:.3e}')
    assert d_merged <= 1e-3 and d_heads <= 1e-3


def test_logits_x3_vs_fp32_device_batch():
    """512 synthetic segments (micro-batch 256, stem + layer1 in SAD_FRONT_MB
    sub-batches of 64 -> every chunk boundary crossed): bf16x3 vs the fp32
    device path, and the decisions they imply."""
    from oracle.decision import interpret_multihead_logits
    from sad import _lib
    from sad.engine import Engine
    sd = merged_sd('n6')
    n = 512
    pcm = torch.empty(n, 128000, dtype=torch.int16, device=DEV)
    _lib.call('sad_synth_pcm', 21, 0, n, 128000, _lib.ptr(pcm), _lib.stream_handle(torch.device(DEV)))
    _, m3 = Engine(sd, DEV, dtype='bf16x3', micro_batch=256).forward_pcm(pcm)
    _, m32 = Engine(sd, DEV, dtype='fp32', micro_batch=128).forward_pcm(pcm)
    torch.cuda.synchronize()
    d = (m3 - m32).abs().max().item()
    print(f'bf16x3 vs fp32 device, {n} segments: max|dlogit| {d:.3e}')
    assert d <= 1e-3
    names = [f'S{i}' for i in range(6)]
    a = [interpret_multihead_logits(r, 0.5, names)[0] for r in m3.cpu()]
    b = [interpret_multihead_logits(r, 0.5, names)[0] for r in m32.cpu()]
    assert a == b


def test_x3_microbatch_invariance():
    from sad import _lib
    from sad.engine import Backbone, FrontEnd, split_merged_state
    _, bases, _ = split_merged_state(merged_sd('n6'))
    pcm = torch.empty(37, 128000, dtype=torch.int16, device=DEV)
    _lib.call('sad_synth_pcm', 3, 0, 37, 128000, _lib.ptr(pcm), _lib.stream_handle(torch.device(DEV)))
    maps = FrontEnd(DEV)(pcm)
    a = Backbone(bases[0], DEV, 'bf16x3', micro_batch=16)(maps)
    b = Backbone(bases[0], DEV, 'bf16x3', micro_batch=37)(maps)
    assert torch.equal(a, b)
