"""CPU: the drop-in model_merger reproduces the reference merger's output
format and key semantics (tests/golden/golden_merger.json, produced by running
the reference's model_merger.main)."""
import csv
import json
import os

import pytest
import torch

from conftest import GOLDEN


def test_merger_matches_reference_semantics(tmp_path):
    from oracle import resnet as ores
    import model_merger as mm
    g = json.load(open(os.path.join(GOLDEN, 'golden_merger.json')))
    torch.manual_seed(123)
    rows = [('m1.pth', 'SynA', 'Real'), ('m2.pth', 'SynB', 'Real'), ('m3.pth', 'SynC', 'Human')]
    heads = {}
    for fn, _, _ in rows:  # trainer checkpoints: unprefixed timm keys + head.* (submodel_trainer.py:707-714)
        tr = ores.create_model('resnet18')
        tr.head = ores.make_head()
        heads[fn] = tr.head[10].bias.detach().clone()
        torch.save({'epoch': 0, 'state_dict': tr.state_dict(), 'best_acc': 50.0}, tmp_path / fn)
    with open(tmp_path / 'm.csv', 'w', newline='') as f:
        w = csv.writer(f)
        w.writerow(['model_filename', 'synthetic_class', 'real_class'])
        w.writerows(rows)
    out = tmp_path / 'merged.pth'
    names = mm.main(['--submodels-folder', str(tmp_path), '--csv-file', str(tmp_path / 'm.csv'),
                     '--output-path', str(out)])
    assert names == g['metadata']['class_names']
    ck = torch.load(out, map_location='cpu', weights_only=True)
    assert sorted(ck.keys()) == g['top_keys']
    assert ck['metadata'] == g['metadata']
    assert len(ck['state_dict']) == g['n_keys']
    keys0 = sorted(k[len('sub_models.0.'):] for k in ck['state_dict'] if k.startswith('sub_models.0.'))
    assert keys0 == g['keys_sub0']
    for j, (fn, _, _) in enumerate(rows):  # heads come from the trainer checkpoints ...
        assert torch.equal(ck['state_dict'][f'sub_models.{j}.head.10.bias'], heads[fn]) == g['head_from_trainer'][j]
    # ... the backbones do not (quirk C2): all sub-models share the constructor's backbone
    tr1 = torch.load(tmp_path / 'm1.pth', weights_only=True)['state_dict']
    assert torch.equal(ck['state_dict']['sub_models.0.base.conv1.weight'], tr1['conv1.weight']) == \
        g['backbone_from_trainer_conv1']
    assert torch.equal(ck['state_dict']['sub_models.0.base.conv1.weight'],
                       ck['state_dict']['sub_models.2.base.conv1.weight'])


def test_merger_real_class_vote():
    import model_merger as mm
    assert mm.merged_real_class(['Real', 'Real']) == 'Real'
    assert mm.merged_real_class(['Real', 'Human', 'Human']) == 'Human'
    assert mm.merged_real_class(['A', 'B']) == 'A'  # Counter.most_common tie -> first seen


def test_merger_empty_csv(tmp_path, capsys):
    import model_merger as mm
    (tmp_path / 'e.csv').write_text('model_filename,synthetic_class,real_class\n')
    assert mm.main(['--submodels-folder', str(tmp_path), '--csv-file', str(tmp_path / 'e.csv'),
                    '--output-path', str(tmp_path / 'x.pth')]) is None
    assert 'No submodels found' in capsys.readouterr().out


@pytest.mark.parametrize('name', ['resnet34', 'resnet50'])
def test_merger_model_name_matches_reference(tmp_path, name):
    """--model-name (model_merger.py:101,129): tests/golden/golden_merger_deep.json
    was written by the reference's model_merger.main with --model-name resnet34 /
    resnet50 (make_golden_deep.py) on trainer checkpoints made the same way."""
    from oracle import resnet as ores
    import model_merger as mm
    g = json.load(open(os.path.join(GOLDEN, 'golden_merger_deep.json')))[name]
    torch.manual_seed(123)
    rows = [('m1.pth', 'SynA', 'Real'), ('m2.pth', 'SynB', 'Real')]
    heads = {}
    for fn, _, _ in rows:
        tr = ores.create_model(name)
        tr.head = ores.make_head(tr.num_features)
        heads[fn] = tr.head[10].bias.detach().clone()
        torch.save({'epoch': 0, 'state_dict': tr.state_dict(), 'best_acc': 50.0}, tmp_path / fn)
    with open(tmp_path / 'm.csv', 'w', newline='') as f:
        w = csv.writer(f)
        w.writerow(['model_filename', 'synthetic_class', 'real_class'])
        w.writerows(rows)
    out = tmp_path / 'merged.pth'
    names = mm.main(['--submodels-folder', str(tmp_path), '--csv-file', str(tmp_path / 'm.csv'),
                     '--output-path', str(out), '--model-name', name])
    assert names == g['metadata']['class_names']
    ck = torch.load(out, map_location='cpu', weights_only=True)
    assert ck['metadata'] == g['metadata'] and len(ck['state_dict']) == g['n_keys']
    assert sorted(k[len('sub_models.0.'):] for k in ck['state_dict'] if k.startswith('sub_models.0.')) == \
        g['keys_sub0']
    assert list(ck['state_dict']['sub_models.0.head.2.weight'].shape) == g['head0_shape']
    for j, (fn, _, _) in enumerate(rows):
        assert torch.equal(ck['state_dict'][f'sub_models.{j}.head.10.bias'], heads[fn]) == g['head_from_trainer'][j]
    tr1 = torch.load(tmp_path / 'm1.pth', weights_only=True)['state_dict']
    assert torch.equal(ck['state_dict']['sub_models.0.base.conv1.weight'], tr1['conv1.weight']) == \
        g['backbone_from_trainer_conv1']
