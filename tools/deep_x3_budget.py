#!/usr/bin/env python3
"""resnet50 in the split-bf16 parity mode (bf16x3): how much of its logit error
against the reference fixture is the split arithmetic itself (VERDICT r4 item
6: the GPU measured 1.05e-3 against a 1e-3 bar, fp32 2.4e-4).

CPU emulation of the device plan (csrc/resnet.hip, dtype bf16x3): BN folded in
float64, rounded to fp32; every weight and every stored activation carried as
hi = bf16(v), lo = bf16(v - hi); each conv = W_hi.X_hi + W_lo.X_hi + W_hi.X_lo
accumulated in fp32 (torch CPU order) or float64; conv3 + the downsample as one
sum, the identity shortcut added in the epilogue (hi + lo); fp32 pool and heads.
Also the same plan with exact fp32 operands (only the accumulation differs from
the fixture) and with the W_lo.X_lo product kept.

Test infrastructure only (imports oracle/).   python tools/deep_x3_budget.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'synthetic-audio-detection_amd'), os.path.join(ROOT, 'tools')]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from deep_bf16_budget import fold  # noqa: E402


def split(v):
    hi = v.to(torch.bfloat16).float()
    lo = (v - hi).to(torch.bfloat16).float()
    return hi, lo


def conv_x3(x, w, b, mode, stride=1, padding=0):
    if mode == 'exact':
        return F.conv2d(x, w, b, stride=stride, padding=padding)
    xh, xl = split(x)
    wh, wl = split(w)
    dt = torch.float64 if mode.endswith('f64') else torch.float32

    def c(a, bb):
        return F.conv2d(a.to(dt), bb.to(dt), None, stride=stride, padding=padding)
    y = c(xh, wh) + c(xh, wl) + c(xl, wh)
    if 'lolo' in mode:
        y = y + c(xl, wl)
    return (y + b.to(dt).view(1, -1, 1, 1)).float()


def store(v, mode):
    if mode == 'exact':
        return v
    h, lo = split(v)
    return h + lo


def features(base, img, mode):
    w, b = fold(base.conv1, base.bn1)
    x = conv_x3(store(img[:, :1], mode), w.sum(1, keepdim=True), b, mode, stride=2, padding=3)
    x = store(F.max_pool2d(F.relu(x), 3, 2, 1), mode)
    for li in range(1, 5):
        for blk in getattr(base, f'layer{li}'):
            w1, b1 = fold(blk.conv1, blk.bn1)
            w2, b2 = fold(blk.conv2, blk.bn2)
            w3, b3 = fold(blk.conv3, blk.bn3)
            t = store(F.relu(conv_x3(x, w1, b1, mode)), mode)
            t = store(F.relu(conv_x3(t, w2, b2, mode, stride=blk.conv2.stride, padding=1)), mode)
            if blk.downsample is not None:
                wd, bd = fold(blk.downsample[0], blk.downsample[1])
                s = blk.downsample[0].stride
                y = conv_x3(torch.cat([t, x[:, :, ::s[0], ::s[1]]], 1), torch.cat([w3, wd], 1), b3 + bd, mode)
            else:
                y = conv_x3(t, w3, b3, mode) + x
            x = store(F.relu(y), mode)
    return x.mean(dim=(2, 3))


def main():
    from oracle import frontend as ofe
    from oracle import resnet as ores
    from sad import weights as sw
    name = sys.argv[1] if len(sys.argv) > 1 else 'resnet50'
    gold = os.path.join(ROOT, 'tests', 'golden')
    sd = sw.merged_state_dict(0, 2, False, bn_stats=sw.load_bn_stats(os.path.join(gold, f'bn_stats_{name}.npz')),
                              model_name=name)
    model = ores.load_merged_state(sd, backbone_name=name)
    fx = dict(np.load(os.path.join(gold, 'golden_deep.npz')))
    pcm = np.load(os.path.join(gold, 'golden_frontend.npz'))['pcm']
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    with torch.no_grad():
        maps = torch.cat([ofe.waveform_to_spectrogram(torch.from_numpy(p.astype(np.float32) / 32768.0), 32000,
                                                      ofe.SpectrogramConfig()) for p in pcm])
        img = ofe.resize_bilinear(maps[:, :1], (512, 512))
        base = model.sub_models[0].base
        ref_h, ref_m = fx[f'{name}_per_head'], fx[f'{name}_merged']

        def heads(feat):
            per = torch.stack([m.head[2:](feat) for m in model.sub_models], 1)
            merged = torch.cat([per[:, :, 1], per[:, :, 0].mean(1, keepdim=True)], 1)
            return per.numpy(), merged.numpy()

        for mode in ('exact', 'x3', 'x3f64', 'x3lolo'):
            h, m = heads(features(base, img, mode))
            print(f'{name} plan {mode:7s}: per-head {np.abs(h - ref_h).max():.3e}  merged {np.abs(m - ref_m).max():.3e}',
                  flush=True)


if __name__ == '__main__':
    main()
