#!/usr/bin/env python3
"""Golden fixture for the trainer hot path, made by running the REFERENCE's own
``train()`` and ``validate()`` (``modular/source/submodel_trainer.py:241-313,
316-385``) on the CPU.

Run only in the build container (it reads /root/reference):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_train.py

The reference module imports torchaudio / torchvision / timm / tensorboard,
which are not installed: stubs are registered as in make_golden.py (timm's
create_model is the in-repo oracle ResNet; SummaryWriter records nothing), then
``submodel_trainer`` is imported unchanged.  The model, optimizer and
scheduler are set up as its ``main()`` does (``:606-660``): timm resnet18
(num_classes=0) + the attached, unused head (quirk C1), everything frozen but
head + layer4, AdamW(filter(requires_grad), lr 1e-3, wd 0.01),
ReduceLROnPlateau(min, 0.5, patience 2); at epoch ``epochs // 3`` layer3 gets
requires_grad after the optimizer was built (``:687-691``, quirk C4).

Data: 4 synthetic "files" x 2 segments (sad.synth seed 13), the val-transform
images of the oracle front end (masks off, crop = the whole image), files 0-3
labelled 0, 1, 1, 0; batch size 2 files -> 2 steps per epoch, 2 epochs (layer3
unfrozen at epoch 1 = 3 // 3 with --epochs 3), then validate() on batch 0.

Recorded per step (the reference's clip_grad_norm_ wrapped to observe it):
loss, pre-clip total norm, clipped grad L2 norms of every layer3/layer4 tensor,
layer4 parameter norms and 64 strided samples after the AdamW step; per epoch:
train() / validate() return values and the learning rate; at the end: every
BatchNorm's running-mean / running-var sums.  Only data is written
(tests/golden/golden_train.json); no reference source or bytecode.
"""
from __future__ import annotations

import json
import os
import sys
import types

import numpy as np
import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'synthetic-audio-detection_amd'))

import make_golden as mg  # noqa: E402
from oracle import resnet as ores  # noqa: E402
from oracle import train as otr  # noqa: E402

FILES = 4
SEED = 13
LABELS = [0, 1, 1, 0]
NOAUG = ((0, 0, 0, 0), (0, 0, 512, 512))


def waves():
    from sad.synth import synth_segment
    return [[torch.from_numpy(synth_segment(SEED, 2 * f + s).astype(np.float32) / 32768.0) for s in range(2)]
            for f in range(FILES)]


def import_reference_trainer():
    mg.install_stubs()
    tb = types.ModuleType('torch.utils.tensorboard')

    class SummaryWriter:
        def __init__(self, *a, **k):
            pass

        def add_scalar(self, *a, **k):
            pass

        def close(self):
            pass

    tb.SummaryWriter = SummaryWriter
    sys.modules['torch.utils.tensorboard'] = tb
    sys.path.insert(0, mg.REF_SRC)
    import submodel_trainer as ref_tr  # noqa
    sys.path.remove(mg.REF_SRC)
    return ref_tr


class _DS:
    classes = ['Real', 'Class1']

    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


class Loader(list):
    def __init__(self, batches, n_files):
        super().__init__(batches)
        self.dataset = _DS(n_files)


def main():
    from sad import train as st
    from sad import weights as sw
    ref_tr = import_reference_trainer()
    wv = waves()
    imgs = [[otr.segment_image(wv[f][s], *NOAUG) for s in range(2)] for f in range(FILES)]
    batches = []
    for b in range(FILES // 2):
        fs = [2 * b, 2 * b + 1]
        batches.append((torch.stack([imgs[f][0] for f in fs]), torch.tensor([LABELS[f] for f in fs]),
                        torch.stack([imgs[f][1] for f in fs]), torch.tensor([LABELS[f] for f in fs])))
    loader = Loader(batches, FILES)
    val_loader = Loader(batches[:1], 2)

    # model / optimizer / scheduler as submodel_trainer.main() (:606-660)
    base_sd = sw.backbone_state_dict(7)
    _, head_sd = st.init_state_dict(42)
    model = ores.create_model('resnet18', pretrained=False, num_classes=0)
    model.load_state_dict(base_sd, strict=True)
    for p in model.parameters():
        p.requires_grad = False
    model.head = ores.make_head(model.num_features)
    model.head.load_state_dict(head_sd, strict=True)
    for p in model.head.parameters():
        p.requires_grad = True
    for p in model.layer4.parameters():
        p.requires_grad = True
    criterion = torch.nn.CrossEntropyLoss()
    optimizer = torch.optim.AdamW(filter(lambda p: p.requires_grad, model.parameters()), lr=1e-3, weight_decay=0.01)
    scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(optimizer, mode='min', factor=0.5, patience=2)

    steps = []
    real_clip = torch.nn.utils.clip_grad_norm_
    l4 = [n for n, _ in model.named_parameters() if n.startswith('layer4.')]
    l3 = [n for n, _ in model.named_parameters() if n.startswith('layer3.')]

    def clip_spy(params, max_norm, *a, **k):
        norm = real_clip(params, max_norm, *a, **k)
        pd = dict(model.named_parameters())
        steps.append({'total_norm': float(norm),
                      'grad_norm': {n: float(pd[n].grad.norm()) for n in l4 + l3 if pd[n].grad is not None}})
        return norm

    torch.nn.utils.clip_grad_norm_ = clip_spy  # train() looks it up through torch.nn.utils (:276)
    args = types.SimpleNamespace()
    epochs_out = []
    total_steps = 0
    epochs = 3
    try:
        for epoch in range(2):
            if epoch == epochs // 3:
                for p in model.layer3.parameters():  # :687-691
                    p.requires_grad = True
            losses = []
            real_ce = criterion.forward

            def ce_spy(out, tgt):
                v = real_ce(out, tgt)
                losses.append(float(v))
                return v
            criterion.forward = ce_spy
            n0 = len(steps)
            eloss, eacc, total_steps = ref_tr.train(args, loader, model, criterion, optimizer, scheduler, epoch,
                                                    types.SimpleNamespace(add_scalar=lambda *a: 0),
                                                    total_steps, torch.device('cpu'))
            criterion.forward = real_ce
            for i, s in enumerate(steps[n0:]):
                s['loss'] = losses[i]
            pd = dict(model.named_parameters())
            steps[-1]['layer4_after'] = {n: {'norm': float(pd[n].detach().norm()), 'sum': float(pd[n].detach().sum()),
                                             'sample': pd[n].detach().flatten()[::max(1, pd[n].numel() // 64)][:64]
                                             .tolist()} for n in l4}
            epochs_out.append({'epoch': epoch, 'train_loss': eloss, 'train_acc': eacc, 'total_steps': total_steps,
                               'lr': optimizer.param_groups[-1]['lr']})
        vloss, vacc, preds, tgts = ref_tr.validate(args, val_loader, model, criterion, 1, torch.device('cpu'))
    finally:
        torch.nn.utils.clip_grad_norm_ = real_clip
    bn = {}
    for n, m in model.named_modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            bn[n] = {'mean_sum': float(m.running_mean.sum()), 'var_sum': float(m.running_var.sum()),
                     'tracked': int(m.num_batches_tracked)}
    out = {'seed_pcm': SEED, 'labels': LABELS, 'base_seed': 7, 'head_seed': 42, 'lr': 1e-3, 'epochs_arg': epochs,
           'steps': steps, 'epochs': epochs_out,
           'validate': {'loss': vloss, 'acc': vacc, 'preds': [int(p) for p in preds], 'targets': [int(t) for t in tgts]},
           'bn_running': bn,
           'layer3_weight_sums': {n: float(dict(model.named_parameters())[n].detach().sum()) for n in l3}}
    with open(os.path.join(HERE, 'golden_train.json'), 'w') as f:
        json.dump(out, f, indent=1)
    for e in epochs_out:
        print(e)
    print('steps', [(round(s['loss'], 6), round(s['total_norm'], 6)) for s in steps])
    print('validate', vloss, vacc, preds)


if __name__ == '__main__':
    main()
