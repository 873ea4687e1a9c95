"""GPU: the drop-in submodel_trainer.py end to end on a tiny synthetic WAV
dataset -- main() through epochs that cross the layer3 unfreeze (quirk C4),
the reference checkpoint format (loadable with weights_only=True, optimizer
state loadable by torch.optim.AdamW over the reference's parameter list,
resume), and the checkpoint feeding the drop-in model_merger and
inference_runner."""
import csv
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _dataset(root, n_train=4, n_test=2):
    from sad import audio as sa
    from sad.synth import synth_labelled_clip
    k = 0
    for mode, n in (('train', n_train), ('test', n_test)):
        for label, cls in enumerate(('Real', 'Class1')):
            d = os.path.join(root, mode, cls)
            os.makedirs(d, exist_ok=True)
            for i in range(n):
                k += 1
                sa.save_pcm16(os.path.join(d, f'{cls}_{i}.wav'), synth_labelled_clip(3, k, label))


def test_trainer_main_checkpoint_merge_infer(tmp_path, monkeypatch):
    import submodel_trainer as smt
    from sad import train as st
    monkeypatch.chdir(tmp_path)
    _dataset(str(tmp_path / 'ds'))
    ck_dir = tmp_path / 'ck'
    best = smt.main(['--data-dir', str(tmp_path / 'ds'), '--epochs', '3', '--batch-size', '2', '--workers', '0',
                     '--checkpoint-dir', str(ck_dir), '--precision', 'fp32', '--Class1', 'SynA'])
    assert 0.0 <= best <= 100.0
    # checkpoint in the reference format, written directly (val accuracy may stay 0)
    base, head = st.init_state_dict(42)
    tr = st.Trainer(base, head, 'cuda:0', 'fp32')
    fe = st.TrainFrontEnd('cuda:0', 'fp32')
    from sad.synth import synth_labelled_clip
    w = torch.stack([torch.from_numpy(synth_labelled_clip(5, i, i % 2)[:128000].astype('float32') / 32768.0)
                     for i in range(4)])
    img = fe(w.to('cuda:0'))
    tr.train_step(img, torch.tensor([0, 1, 0, 1]))
    sched = torch.optim.lr_scheduler.ReduceLROnPlateau(tr.optimizer, mode='min', factor=0.5, patience=2)
    path = ck_dir / 'model_best.pth'
    smt.save_checkpoint(str(path), 0, tr, sched, 50.0, 1)
    ck = torch.load(path, map_location='cpu', weights_only=True)
    assert sorted(ck) == ['best_acc', 'epoch', 'optimizer', 'scheduler', 'state_dict', 'total_steps']
    from oracle import resnet as ores
    from oracle import train as otr
    ref = ores.create_model('resnet18')
    ref.head = ores.make_head()
    assert list(ck['state_dict'].keys()) == list(ref.state_dict().keys())
    ref.load_state_dict(ck['state_dict'], strict=True)
    # the reference's optimizer (filter(requires_grad): layer4 + head) accepts the state
    m, opt = otr.build({k: v for k, v in ck['state_dict'].items() if not k.startswith('head.')},
                       {k[5:]: v for k, v in ck['state_dict'].items() if k.startswith('head.')})
    opt.load_state_dict(ck['optimizer'])
    assert len(opt.state) == len(tr.l4_names)
    # resume into a fresh trainer
    tr2 = st.Trainer(base, head, 'cuda:0', 'fp32')
    tr2.load_state_dict(ck['state_dict'])
    tr2.load_optimizer_state_dict(ck['optimizer'])
    assert tr2.step_count == 1
    assert torch.equal(tr2.m, tr.m) and torch.equal(tr2.net.pflat, tr.net.pflat)
    # merge (model_merger CLI) and run inference (inference_runner CLI) on it
    with open(tmp_path / 'm.csv', 'w', newline='') as f:
        wr = csv.writer(f)
        wr.writerow(['model_filename', 'synthetic_class', 'real_class'])
        wr.writerow(['model_best.pth', 'SynA', 'Real'])
    import model_merger as mm
    names = mm.main(['--submodels-folder', str(ck_dir), '--csv-file', str(tmp_path / 'm.csv'),
                     '--output-path', str(tmp_path / 'merged.pth')])
    assert names == ['SynA', 'Real']
    merged = torch.load(tmp_path / 'merged.pth', map_location='cpu', weights_only=True)
    # quirk C2: the trained head is taken, the trained backbone is not
    assert torch.equal(merged['state_dict']['sub_models.0.head.10.bias'], ck['state_dict']['head.10.bias'])
    from sad import audio as sa
    sa.save_pcm16(str(tmp_path / 'clip.wav'), synth_labelled_clip(9, 0, 1)[:200000])
    import inference_runner as ir
    ir.main(['--merged-model', str(tmp_path / 'merged.pth'), '--audio', str(tmp_path / 'clip.wav'),
             '--output-json', str(tmp_path / 'r.json')])
    import json
    out = json.load(open(tmp_path / 'r.json'))
    assert len(out['segments']) == 1 and set(out['percentages']) == {'SynA', 'Real'}
