#!/usr/bin/env python3
"""Deeper-backbone fixtures written by the REFERENCE's own code.

Run only in the build container (it reads /root/reference, which does not exist
on the GPU box):  ``PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_deep.py``

Same stub scheme as make_golden.py (torchaudio / torchvision / timm restated by
the in-repo oracle; timm.create_model = oracle.resnet.create_model, which
builds timm's resnet34 BasicBlock and resnet50 Bottleneck layouts).  For each
backbone name the reference code runs unchanged:

* ``load_merged_model(path, cpu, backbone_name=name)`` (inference_runner.py:77-123):
  the key mapping, the strict=False load and the dummy forward, then
  ``ModularMultiHeadClassifier`` on the 4 fixture segments' images produced by
  the reference's ``waveform_to_spectrogram`` glue -> merged + per-head logits;
* ``model_merger.main(['--model-name', name, ...])`` (model_merger.py:94-159):
  trainer checkpoints of that backbone + CSV -> merged checkpoint; the key set
  and which tensors came from the trainer files are recorded.

The models are 2 heads on one shared backbone (seed 0, sad.weights), BatchNorm
running statistics calibrated on 12 synthetic segments (train-mode pass of the
oracle, as make_golden.calibrate) and committed as bn_stats_<name>.npz.  Only
data is written: golden_deep.npz, golden_merger_deep.json, bn_stats_*.npz.
"""
from __future__ import annotations

import csv
import io
import json
import os
import sys
import tempfile
from contextlib import redirect_stdout

import numpy as np
import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_golden import fixture_pcm, import_reference  # noqa: E402
from oracle import frontend as ofe  # noqa: E402
from oracle import resnet as ores  # noqa: E402
from sad import weights as sw  # noqa: E402
from sad.synth import synth_segment  # noqa: E402

NAMES = ('resnet34', 'resnet50')
N_HEADS = 2


def calibrate(name, calib_imgs):
    """BN running stats = the statistics of calib_imgs seen by the calibrated
    upstream network (train-mode pass, cumulative momentum), backbone and heads."""
    sd = sw.merged_state_dict(0, N_HEADS, False, model_name=name)
    model = ores.load_merged_state(sd, name)
    for m in model.modules():
        if isinstance(m, (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d)):
            m.momentum = None
            m.reset_running_stats()
    model.train()
    with torch.no_grad():
        feats = model.sub_models[0].base.forward_features(calib_imgs)
        for sm in model.sub_models:
            sm.head(feats)
        for sm in model.sub_models[1:]:
            sm.base.load_state_dict(model.sub_models[0].base.state_dict())
    model.eval()
    return {k: v.numpy().astype(np.float32) for k, v in model.state_dict().items()
            if k.endswith('running_mean') or k.endswith('running_var')}


def main():
    torch.manual_seed(0)
    ref_ir, ref_mm = import_reference()
    pcm = fixture_pcm()
    spec_cfg = ref_ir.SpectrogramConfig(n_fft=2048, hop_length=512, n_mels=128, f_min=20, f_max=12000,
                                        top_db=80, norm='slaney')
    imgs = torch.cat([ref_ir.waveform_to_spectrogram(torch.from_numpy(p.astype(np.float32) / 32768.0), 32000,
                                                     spec_cfg) for p in pcm])
    calib = torch.cat([ofe.waveform_to_spectrogram(torch.from_numpy(synth_segment(99, i).astype(np.float32)
                                                                    / 32768.0), 32000, ofe.SpectrogramConfig())
                       for i in range(12)])
    tmp = tempfile.mkdtemp()
    out, merger = {}, {}
    for name in NAMES:
        stats = calibrate(name, calib)
        np.savez_compressed(os.path.join(HERE, f'bn_stats_{name}.npz'), **stats)
        sd = sw.merged_state_dict(0, N_HEADS, False, bn_stats=stats, model_name=name)
        path = os.path.join(tmp, f'merged_{name}.pth')
        torch.save({'state_dict': sd, 'metadata': {'class_names': ['SyntheticA', 'SyntheticB', 'Real']}}, path)
        with redirect_stdout(io.StringIO()):
            model, _ = ref_ir.load_merged_model(path, torch.device('cpu'), backbone_name=name)
        with torch.no_grad():
            out[f'{name}_merged'] = model(imgs).numpy()
            out[f'{name}_per_head'] = torch.stack([m(imgs) for m in model.sub_models], 1).numpy()
            out[f'{name}_feats0'] = model.sub_models[0].base.forward_features(imgs).mean((2, 3)).numpy()
        print(name, 'merged logits\n', out[f'{name}_merged'])

        # model_merger.main --model-name <name> on trainer-format checkpoints
        torch.manual_seed(123)
        sub_dir = os.path.join(tmp, f'subs_{name}')
        os.makedirs(sub_dir)
        rows = [('m1.pth', 'SynA', 'Real'), ('m2.pth', 'SynB', 'Real')]
        heads = {}
        for fn, _, _ in rows:
            tr = ores.create_model(name)
            tr.head = ores.make_head(tr.num_features)
            heads[fn] = float(tr.head[10].bias.detach().sum())
            torch.save({'epoch': 0, 'state_dict': tr.state_dict(), 'best_acc': 50.0}, os.path.join(sub_dir, fn))
        csv_path = os.path.join(sub_dir, 'm.csv')
        with open(csv_path, 'w', newline='') as f:
            w = csv.writer(f)
            w.writerow(['model_filename', 'synthetic_class', 'real_class'])
            w.writerows(rows)
        outp = os.path.join(tmp, f'merged_mm_{name}.pth')
        old = sys.argv
        sys.argv = ['model_merger.py', '--submodels-folder', sub_dir, '--csv-file', csv_path, '--output-path', outp,
                    '--model-name', name]
        try:
            with redirect_stdout(io.StringIO()):
                ref_mm.main()
        finally:
            sys.argv = old
        mm = torch.load(outp, map_location='cpu', weights_only=True)
        keys = sorted(mm['state_dict'].keys())
        tr1 = torch.load(os.path.join(sub_dir, 'm1.pth'), weights_only=True)['state_dict']
        merger[name] = {
            'metadata': mm['metadata'], 'n_keys': len(keys),
            'keys_sub0': [k[len('sub_models.0.'):] for k in keys if k.startswith('sub_models.0.')],
            'head_from_trainer': [abs(float(mm['state_dict'][f'sub_models.{j}.head.10.bias'].sum()) - heads[r[0]])
                                  < 1e-7 for j, r in enumerate(rows)],
            'backbone_from_trainer_conv1': bool(torch.equal(mm['state_dict']['sub_models.0.base.conv1.weight'],
                                                            tr1['conv1.weight'])),
            'head0_shape': list(mm['state_dict']['sub_models.0.head.2.weight'].shape)}
        print(name, 'merger', merger[name]['metadata'], merger[name]['head_from_trainer'],
              merger[name]['backbone_from_trainer_conv1'], merger[name]['head0_shape'])
    np.savez_compressed(os.path.join(HERE, 'golden_deep.npz'), **out)
    with open(os.path.join(HERE, 'golden_merger_deep.json'), 'w') as f:
        json.dump(merger, f, indent=1)


if __name__ == '__main__':
    main()
