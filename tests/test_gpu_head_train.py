"""GPU: the trainer's --head-loss path (csrc/headtrain.hip) against the CPU
oracle (oracle/train.py head_forward: the reference's model.head of
submodel_trainer.py:613-625 on torch autograd, with the device's dropout masks
restated by head_keep_mask).

Tolerances (fp32 throughout; the head's sums are over <= 2,048 terms):
  * logits and the features' gradient: |d| <= 1e-4 relative to the largest
  * loss: relative <= 1e-5
  * every head parameter gradient: norm-relative <= 1e-4 (the two Linear
    biases feeding BatchNorm have an exact gradient of 0: both sides within
    1e-5 of their weight gradient's norm)
  * BatchNorm1d running statistics after the step: |d| <= 1e-5
  * eval mode (running stats, no dropout): the same as the inference heads
    plan (sad_heads_merge_run) within 1e-5
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize('model_name,B', [('resnet18', 64), ('resnet18', 7), ('resnet50', 32)])
def test_head_train_step_matches_oracle(model_name, B):
    from oracle import train as ot
    from sad import train as st
    base, head = st.init_state_dict(3, model_name)
    g = torch.Generator().manual_seed(5)
    # make the BN affine and running stats non-trivial
    for i, c in ((3, 512), (7, 256)):
        head[f'{i}.weight'] = 1 + 0.2 * torch.randn(c, generator=g)
        head[f'{i}.bias'] = 0.1 * torch.randn(c, generator=g)
        head[f'{i}.running_mean'] = 0.05 * torch.randn(c, generator=g)
        head[f'{i}.running_var'] = 1 + 0.1 * torch.rand(c, generator=g)
    net = st.TrainNet(base, head, DEV, 'fp32', model_name, head_loss=True)
    nf = net.num_features
    feats = torch.rand(B, nf, generator=g) * 2.0
    targets = torch.randint(0, 2, (B,), generator=g)
    seed = 0x1234_5678_9ABC
    fd = feats.to(DEV)
    logits = net.head_forward(fd, True, seed)
    dlog, lc = st.ce_loss(logits, targets, 1.0 / B, want_grad=True)
    dfeat = net.head_backward(fd, dlog, seed)
    torch.cuda.synchronize()

    m = ot.head_module(head, nf)
    f = feats.clone().requires_grad_(True)
    ref = ot.head_forward(m, f, True, seed)
    loss = torch.nn.functional.cross_entropy(ref, targets)
    loss.backward()
    scale = ref.abs().max().item()
    assert (logits.cpu() - ref.detach()).abs().max().item() <= 1e-4 * scale
    assert abs(lc[0].item() / B - loss.item()) <= 1e-5 * abs(loss.item())
    assert (dfeat.cpu() - f.grad).abs().max().item() <= 1e-4 * f.grad.abs().max().item()
    a, b = net.range_head
    gflat = net.gflat[a:b].cpu()
    off = 0
    grads = {}
    for name, shape in st.head_param_layout(nf):
        n = int(torch.Size(shape).numel())
        grads[name] = gflat[off:off + n].view(shape)
        off += n
    for name, g_dev in grads.items():
        gref = dict(m.named_parameters())[name[5:]].grad
        if name in ('head.2.bias', 'head.6.bias'):
            # a Linear bias feeding train-mode BatchNorm: its exact gradient is 0
            # (BN removes the batch mean), both sides hold rounding residue
            wn = grads[name.replace('bias', 'weight')].norm().item()
            assert g_dev.abs().max().item() <= 1e-5 * wn and gref.abs().max().item() <= 1e-5 * wn, name
            continue
        e = _rel(g_dev, gref)
        assert e <= 1e-4, (name, e)
    for i in (3, 7):
        bn = m[i]
        assert (net.head_running[i][0].cpu() - bn.running_mean).abs().max().item() <= 1e-5
        assert (net.head_running[i][1].cpu() - bn.running_var).abs().max().item() <= 1e-5


def test_head_eval_matches_inference_heads():
    """head_forward(train=False) = the inference plan's head on the same weights."""
    from sad import train as st
    from sad.engine import Heads
    base, head = st.init_state_dict(4)
    g = torch.Generator().manual_seed(6)
    for i, c in ((3, 512), (7, 256)):
        head[f'{i}.running_mean'] = 0.05 * torch.randn(c, generator=g)
        head[f'{i}.running_var'] = 1 + 0.1 * torch.rand(c, generator=g)
    net = st.TrainNet(base, head, DEV, 'fp32', head_loss=True)
    feats = (torch.rand(256, 512, generator=g) * 2).to(DEV)
    got = net.head_forward(feats, train=False)
    logits, _ = Heads([head], [0], 1, DEV)([feats])
    torch.cuda.synchronize()
    assert (got - logits[:, 0, :]).abs().max().item() <= 1e-5


def test_trainer_head_loss_learns_synthetic_classes():
    """--head-loss on the synthetic two-class clips (bench_train's data): a
    short bf16 run separates the classes on held-out clips through the head in
    eval mode, which quirk C1's pooled-feature loss cannot (~50 %)."""
    import numpy as np
    from sad import train as st
    from sad.synth import synth_labelled_clip
    torch.manual_seed(0)
    base, head = st.init_state_dict(42)
    tr = st.Trainer(base, head, DEV, 'bf16', lr=1e-3, head_loss=True)
    fe = st.TrainFrontEnd(DEV, 'bf16')
    P = 64
    lab = np.arange(P) % 2
    wav = torch.from_numpy(np.stack([synth_labelled_clip(0, i, int(lab[i]))[:128000] for i in range(P)])
                           .astype(np.float32) / 32768.0).to(DEV)
    t = torch.from_numpy(lab).long()
    g = torch.Generator().manual_seed(1)
    for _ in range(30):
        idx = torch.randperm(P, generator=g)[:32]
        img = fe(wav[idx.to(DEV)])
        loss, c, n, ok = tr.train_step(img, t[idx].to(DEV))
        assert ok
    E = 64
    el = np.arange(E) % 2
    ev = torch.from_numpy(np.stack([synth_labelled_clip(10_000, i, int(el[i]))[:128000] for i in range(E)])
                          .astype(np.float32) / 32768.0).to(DEV)
    feats = tr.net.eval_backbone()(fe.maps(ev))
    _, lc = st.ce_loss(tr.net.head_forward(feats, train=False), torch.from_numpy(el).long())
    acc = lc[1].item() / E
    print(f'--head-loss eval accuracy after 30 steps: {100 * acc:.1f} %')
    assert acc >= 0.9
