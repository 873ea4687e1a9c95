"""GPU: the reference's general model call on [B, 3, 512, 512] tensors whose
channels DIFFER (its load-time check feeds torch.randn(2,3,512,512),
inference_runner.py:119-122, model_merger.py:148-151): the distinct-channel
stem (fp32 conv1 per channel) + the backbone + heads vs the CPU oracle.
Tolerance |dlogit| <= 1e-3 for fp32 and bf16x3; identical-channel input still
takes the folded stem and agrees with the spectrogram path."""
import numpy as np
import pytest
import torch

from conftest import merged_sd

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'


def _model(tag, precision):
    import inference_runner as ir
    from sad.engine import split_merged_state
    sd = merged_sd(tag)
    idx, _, _ = split_merged_state(sd)
    subs = []
    for i in idx:
        sm = ir.BinaryClassifier(init='empty')
        sm.load_state_dict({k[len(f'sub_models.{i}.'):]: v for k, v in sd.items() if k.startswith(f'sub_models.{i}.')},
                           strict=False)
        subs.append(sm)
    return ir.ModularMultiHeadClassifier(subs, DEV, precision, micro_batch=2), sd


@pytest.mark.parametrize('precision', ['fp32', 'bf16x3'])
@pytest.mark.parametrize('tag', ['n6', 'n2'])
def test_distinct_channels_vs_oracle(tag, precision):
    from oracle import resnet as ores
    model, sd = _model(tag, precision)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(3, 3, 512, 512, generator=g)
    out = model(x).cpu()
    with torch.no_grad():
        ref = ores.load_merged_state(sd)(x)
    d = (out - ref).abs().max().item()
    print(f'{tag} {precision} randn(3,3,512,512): max|dlogit| {d:.3e}')
    assert d <= 1e-3


def test_identical_channels_take_folded_stem(golden_frontend):
    from oracle import frontend as ofe
    model, _ = _model('n6', 'fp32')
    maps = torch.from_numpy(golden_frontend['std_map'][:2])
    x = ofe.resize_bilinear(maps.unsqueeze(1), (512, 512)).repeat(1, 3, 1, 1)
    a = model(x).cpu()
    b = model.forward_maps(maps).cpu()
    assert (a - b).abs().max().item() <= 1e-4
    x3 = x.clone()
    x3[:, 2] += 1e-3  # now distinct: the per-channel stem, same function up to the perturbation
    c = model(x3).cpu()
    assert np.isfinite(c.numpy()).all() and (c - a).abs().max().item() <= 5e-2


def test_load_merged_model_runs_reference_dummy_check(tmp_path):
    import inference_runner as ir
    sd = merged_sd('n2')
    p = str(tmp_path / 'm.pth')
    torch.save({'state_dict': sd, 'metadata': {'class_names': ['A', 'B', 'Real']}}, p)
    model, meta = ir.load_merged_model(p, torch.device(DEV))
    assert meta['class_names'] == ['A', 'B', 'Real']
    assert model(torch.randn(2, 3, 512, 512)).shape == (2, 3)
