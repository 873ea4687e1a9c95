"""CPU: host side of the drop-in submodel_trainer.py (no device compute):
CLI defaults, the 2-segment rules, dataset discovery / collate, augmentation
parameter sampling, the timm-order initialisation and checkpoint key layout,
and per-rank sharding."""
import os

import numpy as np
import pytest
import torch


def test_cli_defaults_match_reference():
    import submodel_trainer as smt
    a = smt.parse_args([])
    # submodel_trainer.py:36-52
    assert (a.data_dir, a.batch_size, a.epochs, a.lr, a.workers, a.seed, a.gpu, a.num_gpus) == \
        ('./dataset', 32, 100, 0.001, 20, 42, 0, 1)
    assert (a.checkpoint_dir, a.resume, a.evaluate, a.Class0, a.Class1, a.model_name) == \
        ('./checkpoints', '', False, 'Real', 'Class1', 'resnet18')
    with pytest.raises(SystemExit):
        smt.parse_args(['--model-name', 'vgg16'])


@pytest.mark.parametrize('n,expect', [
    (256000, 'split'), (300000, 'split'), (255999, 'dup'), (128000, 'dup'),
    (127999, 'pad'), (115200, 'pad'), (115199, None), (0, None)])
def test_segment_rules(n, expect):
    """submodel_trainer.py:155-187."""
    import submodel_trainer as smt
    w = torch.arange(n, dtype=torch.float32).reshape(1, -1)
    segs = smt.segment_waveform(w)
    if expect is None:
        assert segs is None
        return
    assert all(s.shape == (1, 128000) for s in segs)
    if expect == 'split':
        assert torch.equal(segs[0][0], w[0, :128000]) and torch.equal(segs[1][0], w[0, 128000:256000])
    elif expect == 'dup':
        assert torch.equal(segs[0], segs[1]) and torch.equal(segs[0][0], w[0, :128000])
    else:
        assert torch.equal(segs[0][0, :n], w[0]) and torch.all(segs[0][0, n:] == 0)


def _write_dataset(root, n_per_class=3, lengths=(256000,)):
    from sad import audio as sa
    from sad.synth import synth_labelled_clip
    k = 0
    for mode in ('train', 'test'):
        for label, cls in enumerate(('Real', 'Class1')):
            d = os.path.join(root, mode, cls)
            os.makedirs(d, exist_ok=True)
            for i in range(n_per_class):
                n = lengths[k % len(lengths)]
                k += 1
                sa.save_pcm16(os.path.join(d, f'c{i}.wav'), synth_labelled_clip(1, k, label, max(n, 1))[:n])


def test_dataset_and_collate(tmp_path):
    import submodel_trainer as smt
    _write_dataset(str(tmp_path), 3, lengths=(256000, 200000, 100000))
    ds = smt.SpectrogramDataset(str(tmp_path), 'train', transform='train', class_names=['Real', 'Class1'])
    assert len(ds) == 6
    assert [t for _, t in ds.samples] == [0, 0, 0, 1, 1, 1]
    items = [ds[i] for i in range(len(ds))]
    assert items[2] is None and items[5] is None  # 100000 < 0.9 * 128000
    s1, t1, s2, t2, aug = items[0]
    assert s1.shape == (128000,) and s2.shape == (128000,) and t1 == t2 == 0
    assert aug.shape == (2, 8) and aug.dtype == torch.int32
    for row in aug.tolist():
        f0, f1, t0, t1_, i, j, h, w = row
        assert 0 <= f0 <= f1 <= 128 and f1 - f0 < 15 and 0 <= t0 <= t1_ <= 251 and t1_ - t0 < 35
        assert 0 <= i and i + h <= 512 and 0 <= j and j + w <= 512
    batch = smt.custom_collate_fn(items)
    assert batch[0].shape == (4, 128000) and batch[4].shape == (4, 2, 8)
    assert smt.custom_collate_fn([None, None]) is None
    val = smt.SpectrogramDataset(str(tmp_path), 'test', transform='val', class_names=['Real', 'Class1'])
    _, _, _, _, aug = val[0]
    assert aug.tolist() == [[0, 0, 0, 0, 0, 0, 512, 512]] * 2
    with pytest.raises(RuntimeError):
        smt.SpectrogramDataset(str(tmp_path), 'nope')


def test_augment_sampling_properties():
    from sad import augment
    g = torch.Generator().manual_seed(0)
    areas, ratios = [], []
    for _ in range(2000):
        i, j, h, w = augment.random_resized_crop_params(generator=g)
        assert 0 <= i <= 512 - h and 0 <= j <= 512 - w
        areas.append(h * w / 512 ** 2)
        ratios.append(w / h)
    assert min(areas) >= 0.79 and max(areas) <= 1.0
    assert min(ratios) >= 0.74 and max(ratios) <= 1.35
    g1, g2 = torch.Generator().manual_seed(5), torch.Generator().manual_seed(5)
    assert augment.specaug_masks(generator=g1) == augment.specaug_masks(generator=g2)


def test_init_state_dict_matches_timm_layout():
    from oracle import resnet as ores
    from sad import train as st
    base, head = st.init_state_dict(42)
    ref = ores.create_model('resnet18')
    ref.head = ores.make_head()
    ref_keys = list(ref.state_dict().keys())
    ours = list(base.keys()) + [f'head.{k}' for k in head.keys()]
    assert ours == ref_keys
    for k, v in ref.state_dict().items():
        got = base[k] if not k.startswith('head.') else head[k[5:]]
        assert got.shape == v.shape, k
    # timm init: kaiming_normal_(fan_out, relu) convs, zero_init_last bn2.weight
    w = base['layer3.0.conv2.weight']
    assert abs(w.std().item() - (2.0 / (256 * 9)) ** 0.5) < 0.02 * (2.0 / (256 * 9)) ** 0.5
    assert all(torch.all(base[f'{p}.bn2.weight'] == 0) for p, *_ in st.BLOCKS)
    assert torch.all(base['bn1.weight'] == 1)
    b2, _ = st.init_state_dict(42)
    assert all(torch.equal(base[k], b2[k]) for k in base)
    # trainable set = layer4 (the head gets no gradient, quirk C1)
    names = [n for n, _ in st.param_layout()]
    assert sum(int(np.prod(s)) for n, s in st.param_layout() if n.startswith('layer4.')) == 8_393_728
    assert names[-1] == 'layer4.1.bn2.bias'


def test_rank_sharding_is_disjoint(tmp_path):
    import submodel_trainer as smt
    _write_dataset(str(tmp_path), 5)
    args = smt.parse_args(['--data-dir', str(tmp_path), '--batch-size', '2', '--workers', '0'])
    seen = []
    for r in range(2):
        tl, vl = smt.get_dataloaders(args, rank=r, world=2)
        tl.sampler.set_epoch(0)
        idx = list(iter(tl.sampler))
        seen.append(set(idx))
        assert tl.batch_size == 2
    assert not (seen[0] & seen[1]) and len(seen[0] | seen[1]) == 10


def test_labelled_clips_differ_by_class():
    from sad.synth import synth_labelled_clip
    a = synth_labelled_clip(0, 1, 0).astype(np.float64)
    b = synth_labelled_clip(0, 1, 1).astype(np.float64)
    assert a.shape == b.shape == (256000,)
    # class 1 = harmonic stack: a dominant spectral line; class 0 = coloured noise: none
    fa, fb = np.abs(np.fft.rfft(a)) ** 2, np.abs(np.fft.rfft(b)) ** 2
    assert fb.max() / fb.mean() > 1000 > fa.max() / fa.mean()
