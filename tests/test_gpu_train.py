"""GPU parity of the trainer hot path (submodel_trainer.py)
against the CPU oracle (oracle/train.py, torch autograd fp32).

Tolerances (fp32 parity mode unless stated):
  * train front end (SpecAugment + standardise + resize + RandomResizedCrop):
    max |d| <= 5e-4 on the standardised 512x512 image
  * train-mode forward (batch-statistics BN): pooled features relative <= 1e-4,
    BN running stats after the step relative <= 1e-4
  * step: loss relative <= 1e-4; total grad norm relative <= 1e-3; clipped
    gradients per tensor norm-relative <= 5e-3 (fp32 summation order through up
    to four BN backward passes; ReLU masks at |x| ~ 0), BN bias gradients
    <= 8e-3 (``_bar``); parameters after AdamW
    |d| <= 1e-6 + 1e-2 * lr where the oracle's gradient is not negligible
    (AdamW's first steps move a weight by ~lr*sign(g))
  * quirk C4 (layer3 unfrozen, never zeroed, not stepped): accumulated layer3
    gradients norm-relative <= 5e-3, layer3 weights bit-identical
  * bf16 throughput mode: loss relative <= 3e-2, gradient cosine >= 0.98
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'


def _bar(name: str) -> float:
    """Per-tensor gradient bar: 5e-3, and 8e-3 for BatchNorm biases.  A BN
    bias gradient is the sum of dy over every pixel of the batch, ~1e-4 in
    magnitude from thousands of near-cancelling terms, so rounding-level input
    changes move it most: layer4.1.bn1.bias of resnet34 came out at 5.3e-3
    when the trainer's front end moved onto torchaudio's fp32 filterbank
    (round 5), layer4.0.bn1.bias of resnet18's second step at 5.6e-3 when one
    power bin's summation order changed (round 6).  Every other tensor holds
    5e-3."""
    return 8e-3 if '.bn' in name and name.endswith('.bias') else 5e-3


def _waves(n):
    fx = np.load(os.path.join(GOLDEN, 'golden_frontend.npz'))
    pcm = fx['pcm'][:n].astype(np.float32) / 32768.0
    return torch.from_numpy(pcm)


def _aug(n, seed=3):
    from sad import augment
    g = torch.Generator().manual_seed(seed)
    masks = [augment.specaug_masks(generator=g) for _ in range(n)]
    boxes = [augment.random_resized_crop_params(generator=g) for _ in range(n)]
    return masks, boxes


@pytest.fixture(scope='module')
def model_sd():
    from sad import train as st
    from sad import weights as sw
    base = sw.backbone_state_dict(7)  # non-degenerate BN weights (timm's zero_init_last would zero bn2)
    _, head = st.init_state_dict(42)
    return base, head


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def test_train_frontend_vs_oracle():
    from oracle import train as otr
    from sad.train import TrainFrontEnd
    n = 4
    w = _waves(n)
    masks, boxes = _aug(n)
    fe = TrainFrontEnd(DEV, 'fp32')
    img = fe(w.to(DEV), torch.tensor(masks, dtype=torch.int32), torch.tensor(boxes, dtype=torch.int32)).cpu()
    for i in range(n):
        ref = otr.segment_image(w[i], masks[i], boxes[i])
        assert torch.equal(ref[0], ref[1]) and torch.equal(ref[0], ref[2])
        d = (img[i] - ref[0]).abs().max().item()
        print(f'seg {i} mask {masks[i]} box {boxes[i]}: max|d| = {d:.3e}')
        assert d <= 5e-4
    # val transform: no masks, Resize only
    img = fe(w.to(DEV)).cpu()
    ref = otr.segment_image(w[0])
    assert (img[0] - ref[0]).abs().max().item() <= 5e-4


def _oracle_inputs(img):
    return img.float().cpu().unsqueeze(1).repeat(1, 3, 1, 1)


def test_train_forward_fp32(model_sd):
    from oracle import train as otr
    from sad.train import TrainNet
    base, head = model_sd
    n = 4
    w = _waves(n)
    from sad.train import TrainFrontEnd
    img = TrainFrontEnd(DEV, 'fp32')(w.to(DEV))
    net = TrainNet(base, head, DEV, 'fp32')
    feats, _ = net.forward_train(img)
    torch.cuda.synchronize()
    m, _ = otr.build(base, head)
    m.train()
    with torch.no_grad():
        ref = m(_oracle_inputs(img))
    r = _rel(feats.cpu(), ref)
    print(f'train-mode features rel err {r:.3e}')
    assert r <= 1e-4
    sd = net.base_state_dict()
    for k in ('bn1', 'layer1.0.bn1', 'layer3.0.downsample.1', 'layer4.1.bn2'):
        bn = m.base.get_submodule(k)
        r1 = _rel(sd[f'{k}.running_mean'], bn.running_mean)
        r2 = _rel(sd[f'{k}.running_var'], bn.running_var)
        assert r1 <= 1e-4 and r2 <= 1e-4, (k, r1, r2)
        assert int(sd[f'{k}.num_batches_tracked']) == int(bn.num_batches_tracked)


def _run_steps(model_sd, dtype, n_steps, unfreeze_at=None, lr=1e-3, sync=True, model_name='resnet18'):
    """n_steps of the device trainer and the oracle on the same batch.  With
    ``sync`` the oracle's layer4 weights are reset to the device's before every
    step after the first, so each step's gradients are compared from identical
    weights (AdamW's ~lr*sign(g) update would otherwise amplify fp32 rounding
    differences of near-zero gradients into weight differences)."""
    from oracle import train as otr
    from sad.train import Trainer, TrainFrontEnd
    base, head = model_sd
    n = 4
    w = _waves(n)
    fe = TrainFrontEnd(DEV, dtype)
    img = fe(w.to(DEV))
    targets = torch.tensor([0, 1, 1, 0])
    tr = Trainer(base, head, DEV, dtype, lr=lr, model_name=model_name)
    m, opt = otr.build(base, head, lr=lr, model_name=model_name)
    x_ref = _oracle_inputs(img)
    out = []
    for step in range(n_steps):
        if unfreeze_at is not None and step == unfreeze_at:
            tr.unfreeze_layer3()
            otr.unfreeze_layer3(m)
        if sync and step > 0:
            with torch.no_grad():
                for name, p in m.base.named_parameters():
                    if name.startswith('layer4.'):
                        p.copy_(tr.net.params[name].cpu())
        loss, correct, tot, ok = tr.train_step(img, targets, n)
        torch.cuda.synchronize()
        rloss, routs, rnorm = otr.train_step(m, opt, x_ref, targets)
        g = {name: tr.net.grads[name].cpu() for name, _ in m.base.named_parameters()
             if name.startswith(('layer3.', 'layer4.'))}
        rg = {name: p.grad.clone() for name, p in m.base.named_parameters() if p.grad is not None}
        out.append(dict(loss=loss, rloss=rloss.item(), norm=tr.last_norm.cpu(), rnorm=rnorm.item(), g=g, rg=rg))
        assert ok
    return tr, m, out


def test_train_step_fp32(model_sd):
    lr = 1e-3
    tr, m, out = _run_steps(model_sd, 'fp32', 1, lr=lr)
    o = out[0]
    print(f"loss {o['loss']:.6f} vs {o['rloss']:.6f}; norm {o['norm'][0]:.6f} vs {o['rnorm']:.6f}")
    assert abs(o['loss'] - o['rloss']) <= 1e-4 * abs(o['rloss'])
    assert abs(o['norm'][0].item() - o['rnorm']) <= 1e-3 * o['rnorm']
    net = tr.net
    for name, p in m.base.named_parameters():
        if not name.startswith('layer4.'):
            assert p.grad is None
            continue
        g_ref = o['rg'][name]
        r = _rel(o['g'][name], g_ref)
        assert r <= _bar(name), (name, r)
        # parameters after the AdamW step
        d = (net.params[name].cpu() - p.detach()).abs()
        big = g_ref.abs() > 1e-3 * g_ref.abs().max()
        tol = 1e-6 + 1e-2 * lr
        frac_bad = (d[big] > tol).float().mean().item() if big.any() else 0.0
        print(f'{name:32s} grad rel {r:.2e}  param mismatch frac {frac_bad:.2e}')
        assert frac_bad <= 1e-3, (name, frac_bad, d.max().item())
    # running stats of a frozen layer and a trained one
    sd = net.base_state_dict()
    for k in ('layer2.1.bn1', 'layer4.0.downsample.1'):
        bn = m.base.get_submodule(k)
        assert _rel(sd[f'{k}.running_var'], bn.running_var) <= 1e-4


def test_train_three_steps_fp32(model_sd):
    tr, m, out = _run_steps(model_sd, 'fp32', 3)
    for i, o in enumerate(out):
        print(f"step {i}: loss {o['loss']:.6f} vs {o['rloss']:.6f}; norm {o['norm'][0]:.6f} vs {o['rnorm']:.6f}")
        assert abs(o['loss'] - o['rloss']) <= 1e-4 * abs(o['rloss'])
        assert abs(o['norm'][0].item() - o['rnorm']) <= 1e-3 * o['rnorm']
        for name, gr in o['rg'].items():
            assert _rel(o['g'][name], gr) <= _bar(name), (i, name)


def test_train_step_layer3_quirk_c4(model_sd):
    """layer3 unfrozen after the optimizer was built: its grads accumulate over
    steps (never zeroed), enter the clip norm (and are scaled by it), and the
    weights never move."""
    tr, m, out = _run_steps(model_sd, 'fp32', 3, unfreeze_at=1)
    net = tr.net
    for i, o in enumerate(out):
        print(f"step {i}: norm {o['norm'][0]:.6f} vs {o['rnorm']:.6f}")
        assert abs(o['norm'][0].item() - o['rnorm']) <= 1e-3 * o['rnorm'], (i, o['norm'], o['rnorm'])
        has3 = any(k.startswith('layer3.') for k in o['rg'])
        assert has3 == (i >= 1)
        for name, gr in o['rg'].items():
            assert _rel(o['g'][name], gr) <= _bar(name), (i, name, _rel(o['g'][name], gr))
    for name, p in m.base.named_parameters():
        if name.startswith('layer3.'):
            assert torch.equal(net.params[name].cpu(), p.detach())  # not stepped


def test_train_step_bf16(model_sd):
    tr, m, out = _run_steps(model_sd, 'bf16', 1)
    o = out[0]
    print(f"bf16 loss {o['loss']:.5f} vs fp32 oracle {o['rloss']:.5f}")
    assert abs(o['loss'] - o['rloss']) <= 3e-2 * abs(o['rloss'])
    g = torch.cat([tr.net.grads[n].cpu().flatten() for n in tr.l4_names])
    gr = torch.cat([p.grad.flatten() for n, p in m.base.named_parameters() if n.startswith('layer4.')])
    cos = torch.nn.functional.cosine_similarity(g.double(), gr.double(), dim=0).item()
    print(f'bf16 layer4 gradient cosine vs oracle: {cos:.5f}')
    assert cos >= 0.98


def test_train_ddp_matches_single_process_math(model_sd):
    """The all-reduce path's arithmetic on one rank: a batch of 4 split as 2
    'replicas' (each with its own BN statistics) and gradients summed equals
    two half-batch forwards with loss scale 1/4 -- checked against the oracle's
    DataParallel semantics (per-replica BN) on CPU."""
    from oracle import train as otr
    from sad.train import Trainer, TrainFrontEnd
    base, head = model_sd
    w = _waves(4)
    img = TrainFrontEnd(DEV, 'fp32')(w.to(DEV))
    targets = torch.tensor([0, 1, 1, 0])
    net = Trainer(base, head, DEV, 'fp32').net
    g_sum = None
    from sad.train import ce_loss
    for half in (slice(0, 2), slice(2, 4)):
        feats, saved = net.forward_train(img[half].contiguous())
        d, _ = ce_loss(feats, targets[half], 1.0 / 4, want_grad=True)
        net.backward(d, saved)
        g = net.gflat[net.range4[0]:net.range4[1]].clone()
        g_sum = g if g_sum is None else g_sum + g
    torch.cuda.synchronize()
    # oracle: two replicas, each BN over its half; grads of the global mean
    m, _ = otr.build(base, head)
    m.train()
    x = _oracle_inputs(img)
    outs = torch.cat([m(x[0:2]), m(x[2:4])])
    torch.nn.CrossEntropyLoss()(outs, targets).backward()
    gr = torch.cat([p.grad.flatten() for n, p in m.base.named_parameters() if n.startswith('layer4.')])
    assert _rel(g_sum.cpu(), gr) <= 5e-3


def test_train_step_resnet34_fp32():
    """--model-name resnet34 (BasicBlock, layers 3-4-6-3) on the same trainer
    kernels: one step's loss, clip norm and layer4 gradients vs autograd."""
    from sad import train as st
    from sad import weights as sw
    sd = (sw.backbone_state_dict(7, 'resnet34'), st.init_state_dict(42)[1])
    tr, m, out = _run_steps(sd, 'fp32', 1, model_name='resnet34')
    o = out[0]
    print(f"resnet34 loss {o['loss']:.6f} vs {o['rloss']:.6f}; norm {o['norm'][0]:.6f} vs {o['rnorm']:.6f}")
    assert abs(o['loss'] - o['rloss']) <= 1e-4 * abs(o['rloss'])
    assert abs(o['norm'][0].item() - o['rnorm']) <= 1e-3 * o['rnorm']
    assert set(o['rg']) == {n for n in o['g'] if n.startswith('layer4.')}
    for name, gr in o['rg'].items():
        assert _rel(o['g'][name], gr) <= _bar(name), name
    assert len([b for b in tr.net.blocks if b[0].startswith('layer3.')]) == 6


def test_train_step_resnet34_layer3_unfrozen_fp32():
    """resnet34 with layer3 unfrozen (quirk C4): backward through layer3's 6
    BasicBlocks and the stride-2 dgrad into layer3.0; the accumulated layer3
    gradients vs autograd, norm-relative 1e-2 (a layer3 gradient crosses up to
    16 BN backward passes here; resnet18's tests hold 5e-3 over <= 8)."""
    from sad import train as st
    from sad import weights as sw
    sd = (sw.backbone_state_dict(7, 'resnet34'), st.init_state_dict(42)[1])
    tr, m, out = _run_steps(sd, 'fp32', 1, unfreeze_at=0, model_name='resnet34')
    o = out[0]
    assert abs(o['loss'] - o['rloss']) <= 1e-4 * abs(o['rloss'])
    assert abs(o['norm'][0].item() - o['rnorm']) <= 1e-3 * o['rnorm']
    l3 = [n for n in o['rg'] if n.startswith('layer3.')]
    assert len(l3) == len([n for n in tr.net.names if n.startswith('layer3.')])
    worst = 0.0
    for name in l3:  # the step's layer3 grads, folded into the never-zeroed .grad and clipped (C4)
        e = _rel(o['g'][name], o['rg'][name])
        worst = max(worst, e)
        assert e <= 1e-2, (name, e)
    print(f'resnet34 layer3 grads (unfrozen): worst norm-rel {worst:.2e} over {len(l3)} tensors')


def test_train_step_resnet50_fp32():
    """--model-name resnet50 (Bottleneck, 3-4-6-3): the Bottleneck forward /
    backward on the same trainer kernels (1x1 convs, stride on the 3x3, the
    downsample as 1x1/s + BN): one step's loss, clip norm and layer4 gradients
    vs autograd; then a step with layer3 unfrozen (strided 3x3 dgrad into
    layer3, quirk C4)."""
    from sad import train as st
    from sad import weights as sw
    sd = (sw.backbone_state_dict(7, 'resnet50'), st.init_state_dict(42, 'resnet50')[1])
    tr, m, out = _run_steps(sd, 'fp32', 2, unfreeze_at=1, model_name='resnet50')
    for k, o in enumerate(out):
        print(f"resnet50 step {k}: loss {o['loss']:.6f} vs {o['rloss']:.6f}; "
              f"norm {o['norm'][0]:.6f} vs {o['rnorm']:.6f}")
        assert abs(o['loss'] - o['rloss']) <= 1e-4 * abs(o['rloss'])
        assert abs(o['norm'][0].item() - o['rnorm']) <= 1e-3 * o['rnorm']
        # fp32 summation-order error grows with the BN backward passes a
        # gradient crosses (3 per Bottleneck, batch of 4 -> 1024 values per layer4
        # BN channel): layer4.2 <= 1e-2, .1 <= 2e-2, .0 <= 3e-2 (measured <= 1.1e-2)
        tol = {'layer4.2': 1e-2, 'layer4.1': 2e-2, 'layer4.0': 3e-2}
        for name, gr in o['rg'].items():
            if name.startswith('layer4.'):
                assert _rel(o['g'][name], gr) <= tol[name[:8]], name
    assert set(out[0]['rg']) == {n for n in out[0]['g'] if n.startswith('layer4.')}
    assert tr.net.bottleneck and tr.net.num_features == 2048


def test_train_step_resnet50_bf16_runs():
    """bf16 throughput mode on Bottlenecks vs the fp32 oracle: loss within 3e-2,
    and the layer4 gradients' cosine per block.  bf16 activation rounding is
    amplified by every BN backward pass a gradient crosses (3 per Bottleneck), so
    the bound loosens with depth: layer4.2 >= 0.9, the whole of layer4 >= 0.6
    (measured 0.93 / 0.70 / 0.62 for layer4.2 / .1 / .0; the forward's pooled
    features are already ~7e-2 from fp32 in bf16 on resnet50)."""
    from sad import train as st
    from sad import weights as sw
    sd = (sw.backbone_state_dict(7, 'resnet50'), st.init_state_dict(42, 'resnet50')[1])
    tr, m, out = _run_steps(sd, 'bf16', 1, model_name='resnet50')
    o = out[0]
    assert abs(o['loss'] - o['rloss']) <= 3e-2 * abs(o['rloss'])

    def cos(names):
        g = torch.cat([o['g'][n].flatten() for n in names]).double()
        gr = torch.cat([o['rg'][n].flatten() for n in names]).double()
        return torch.nn.functional.cosine_similarity(g, gr, dim=0).item()
    per = {b: cos([n for n in sorted(o['rg']) if n.startswith(b)]) for b in ('layer4.2', 'layer4.1', 'layer4.0')}
    total = cos(sorted(o['rg']))
    print(f'resnet50 bf16 loss {o["loss"]:.5f} vs {o["rloss"]:.5f}; layer4 grad cosine {total:.4f}, per block '
          + ', '.join(f'{b} {c:.4f}' for b, c in per.items()))
    assert per['layer4.2'] >= 0.9 and total >= 0.6


def _cosines(o, prefix='layer4.'):
    return {n: torch.nn.functional.cosine_similarity(o['g'][n].flatten().double(), gr.flatten().double(),
                                                     dim=0).item()
            for n, gr in o['rg'].items() if n.startswith(prefix)}


def test_train_step_resnet50_mixed_gradient_gate():
    """--precision mixed (sad.train.MixedNet: stem + layers 1-3 in fp32, layer4
    in bf16, forward and backward) is the bf16 trainer whose gradients track
    fp32 autograd: EVERY layer4 parameter tensor's gradient cosine >= 0.95 on
    resnet50 (bf16 throughput mode: 0.93 / 0.70 / 0.62 per block; the CPU
    emulation of the mixed arithmetic, tools/bf16_grad_emulation.py, gives a
    per-tensor minimum of 0.983), loss within 1e-2; then a step with layer3
    unfrozen (quirk C4: its gradient crosses back from the bf16 layer4 into the
    fp32 layer3 through sad_cast_run) with the same bar on layer3's tensors."""
    from sad import train as st
    from sad import weights as sw
    sd = (sw.backbone_state_dict(7, 'resnet50'), st.init_state_dict(42, 'resnet50')[1])
    tr, m, out = _run_steps(sd, 'mixed', 2, unfreeze_at=1, model_name='resnet50')
    assert isinstance(tr.net, st.MixedNet)
    for k, o in enumerate(out):
        c4 = _cosines(o, 'layer4.')
        c3 = _cosines(o, 'layer3.')
        worst = min(c4.items(), key=lambda kv: kv[1])
        print(f"resnet50 mixed step {k}: loss {o['loss']:.5f} vs {o['rloss']:.5f}; layer4 min per-tensor cosine "
              f"{worst[1]:.4f} ({worst[0]})" + (f"; layer3 min {min(c3.values()):.4f}" if c3 else ''))
        assert abs(o['loss'] - o['rloss']) <= 1e-2 * abs(o['rloss'])
        assert len(c4) == len([n for n in tr.net.names if n.startswith('layer4.')])
        assert worst[1] >= 0.95, worst
        assert (len(c3) > 0) == (k >= 1)
        if c3:
            assert min(c3.values()) >= 0.95, min(c3.items(), key=lambda kv: kv[1])
    # the frozen prefix is never stepped; layer4 moved
    for name, p in m.base.named_parameters():
        if name.startswith('layer3.'):
            assert torch.equal(tr.net.params[name].cpu(), p.detach())


def test_train_step_resnet18_mixed(model_sd):
    """resnet18 in the mixed precision: loss within 1e-3 relative of autograd and
    every layer4 tensor's gradient cosine >= 0.99; running statistics of the
    fp32 prefix as fp32's (<= 1e-4)."""
    tr, m, out = _run_steps(model_sd, 'mixed', 1)
    o = out[0]
    c4 = _cosines(o)
    print(f"resnet18 mixed loss {o['loss']:.6f} vs {o['rloss']:.6f}; min cosine {min(c4.values()):.5f}")
    assert abs(o['loss'] - o['rloss']) <= 1e-3 * abs(o['rloss'])
    assert min(c4.values()) >= 0.99
    sd = tr.net.base_state_dict()
    for k in ('layer2.1.bn1', 'layer3.0.downsample.1'):
        bn = m.base.get_submodule(k)
        assert _rel(sd[f'{k}.running_var'], bn.running_var) <= 1e-4
