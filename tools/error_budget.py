#!/usr/bin/env python3
"""Per-layer error budget of the bf16 plan (CPU emulation).

Emulates the device plan's arithmetic on the CPU for ResNet-18 (BN folded into
each conv in float64, conv2 + shortcut as one sum, fp32 accumulation, fused
average pool, fp32 heads) with three independent switches per conv:

  * W: the conv's folded weights rounded to bf16 (else fp32);
  * X: the conv's output activation rounded to bf16 (else fp32);
  * the stem's LDS image band rounded to bf16 (stem input).

and reports max|dlogit| of the merged [B, N+1] logits against the all-fp32
emulation, over the 16 reference-fixture segments and model n6 (the bench's
6-head ensemble).  Rows: all bf16 (the throughput mode), weights only,
activations only, then one conv in bf16 with the rest fp32, and the cumulative
tails (bf16 from conv i on).  The conclusion goes to DESIGN.md section 3b.

Test infrastructure only (imports oracle/).  python tools/error_budget.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'synthetic-audio-detection_amd'), os.path.join(ROOT, 'tests', 'golden')]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def _bf(x):
    return x.to(torch.bfloat16).float()


def fold(conv, bn):
    s = bn.weight.double() / torch.sqrt(bn.running_var.double() + 1e-5)
    w = (conv.weight.double() * s.view(-1, 1, 1, 1)).float()
    b = (bn.bias.double() - bn.running_mean.double() * s).float()
    return w, b


def conv_names():
    names = ['stem']
    for li in range(1, 5):
        for bi in range(2):
            names += [f'l{li}.{bi}.c1', f'l{li}.{bi}.c2']
    return names


def features(base, img, wbf, xbf, img_bf=True):
    """Pooled features under per-conv rounding sets wbf / xbf (conv names)."""
    rw = lambda n, w: _bf(w) if n in wbf else w  # noqa: E731
    rx = lambda n, x: _bf(x) if n in xbf else x  # noqa: E731
    w, b = fold(base.conv1, base.bn1)
    x0 = _bf(img[:, :1]) if img_bf else img[:, :1]
    x = F.conv2d(x0, rw('stem', w.sum(1, keepdim=True)), b, stride=2, padding=3)
    x = rx('stem', F.max_pool2d(F.relu(x), 3, 2, 1))
    for li in range(1, 5):
        for bi, blk in enumerate(getattr(base, f'layer{li}')):
            n1, n2 = f'l{li}.{bi}.c1', f'l{li}.{bi}.c2'
            w1, b1 = fold(blk.conv1, blk.bn1)
            w2, b2 = fold(blk.conv2, blk.bn2)
            t = rx(n1, F.relu(F.conv2d(x, rw(n1, w1), b1, stride=blk.conv1.stride, padding=1)))
            y = F.conv2d(t, rw(n2, w2), b2, padding=1)
            if blk.downsample is not None:
                wd, bd = fold(blk.downsample[0], blk.downsample[1])
                y = y + F.conv2d(x, rw(n2, wd), bd, stride=blk.downsample[0].stride)
            else:
                y = y + x
            y = F.relu(y)
            # the last conv's map is never stored: the fused pool sums fp32
            x = y if (li == 4 and bi == 1) else rx(n2, y)
    return x.mean(dim=(2, 3))


def merged(model, feat):
    real, syn = [], []
    for m in model.sub_models:
        o = m.head[2:](feat)
        real.append(o[:, 0:1])
        syn.append(o[:, 1:2])
    return torch.cat([torch.cat(syn, 1), torch.cat(real, 1).mean(1, keepdim=True)], 1)


def main():
    from make_golden_models16 import segments16
    from oracle import frontend as ofe
    from oracle import resnet as ores
    from sad import weights as sw
    gold = os.path.join(ROOT, 'tests', 'golden')
    sd = sw.merged_state_dict(0, 6, False, bn_stats=sw.load_bn_stats(os.path.join(gold, 'bn_stats_n6.npz')))
    model = ores.load_merged_state(sd)
    pcm = segments16()
    with torch.no_grad():
        maps = torch.cat([ofe.waveform_to_spectrogram(torch.from_numpy(p.astype(np.float32) / 32768.0), 32000,
                                                      ofe.SpectrogramConfig()) for p in pcm])
        img = maps if maps.shape[-1] == 512 else ofe.resize_bilinear(maps[:, :1], (512, 512))
        base = model.sub_models[0].base
        names = conv_names()
        allset = set(names)
        ref = merged(model, features(base, img, set(), set(), img_bf=False))
        fx = np.load(os.path.join(gold, 'golden_models16.npz'))
        print(f'fp32 emulation vs reference fixture: {np.abs(ref.numpy() - fx["n6_merged"]).max():.3e}')

        def row(tag, wbf, xbf, img_bf=True):
            out = merged(model, features(base, img, wbf, xbf, img_bf))
            d = (out - ref).abs().max().item()
            print(f'{tag:34s} max|dlogit| {d:.3e}', flush=True)
            return d

        row('all bf16 (throughput mode)', allset, allset)
        row('weights bf16, activations fp32', allset, set(), img_bf=False)
        row('activations bf16, weights fp32', set(), allset)
        row('stem image band bf16 only', set(), set(), img_bf=True)
        for n in names:
            row(f'only {n} bf16 (W+X)', {n}, {n}, img_bf=(n == 'stem'))
        for n in names:
            row(f'only {n} weights bf16', {n}, set(), img_bf=False)
        for i, n in enumerate(names):
            tail = set(names[i:])
            row(f'bf16 from {n} on', tail, tail, img_bf=(i == 0))


if __name__ == '__main__':
    main()
