"""CPU: pin the oracle against the reference-generated fixtures and against
independent float64 implementations (numpy FFT, transformers' mel bank and
ResNet)."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, merged_sd


def test_mel_fbank_vs_transformers():
    from transformers.audio_utils import mel_filter_bank
    from oracle import frontend as ofe
    for norm in ('slaney', None):
        fb = ofe.melscale_fbanks(1025, 20.0, 12000.0, 128, 32000, norm).numpy()
        ref = mel_filter_bank(num_frequency_bins=1025, num_mel_filters=128, min_frequency=20.0, max_frequency=12000.0,
                              sampling_rate=32000, norm=norm, mel_scale='htk')
        assert np.abs(fb - ref).max() <= 2e-5 * max(1.0, np.abs(ref).max())
        assert (fb > 0).sum() == (ref > 0).sum() == 1515


def test_stft_power_vs_numpy():
    from oracle import frontend as ofe
    from sad.synth import synth_segment
    x = synth_segment(3, 1).astype(np.float64) / 32768.0
    p = ofe.power_spectrogram(torch.from_numpy(x.astype(np.float32))).numpy()
    xp = np.pad(x, 1024, mode='reflect')
    w = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(2048) / 2048)
    fr = np.stack([xp[i * 512:i * 512 + 2048] * w for i in range(251)])
    ref = (np.abs(np.fft.rfft(fr, axis=1)) ** 2).T
    assert p.shape == (1025, 251)
    assert np.abs(p - ref).max() <= 1e-6 * ref.max()


def test_oracle_frontend_reproduces_golden(golden_frontend):
    from oracle import frontend as ofe
    db, m = ofe.batch_maps(golden_frontend['pcm'])
    assert np.abs(db.numpy() - golden_frontend['mel_db']).max() <= 1e-5
    assert np.abs(m.numpy() - golden_frontend['std_map']).max() <= 1e-6
    img = ofe.resize_bilinear(m.unsqueeze(1), (512, 512))[:, 0].double()
    assert np.abs(img.sum(2).numpy() - golden_frontend['img_rowsum']).max() <= 1e-6


def test_oracle_resnet_vs_transformers_topology():
    """The timm-named restatement computes the same function as an independent
    BasicBlock ResNet implementation (transformers.ResNetModel) given the same
    weights -- pins conv/BN/shortcut/pool ordering (timm is not installed)."""
    from transformers import ResNetConfig, ResNetModel
    from oracle import resnet as ores
    torch.manual_seed(0)
    ours = ores.ResNet().eval()
    for mod in ours.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.running_mean.uniform_(-0.1, 0.1)
            mod.running_var.uniform_(0.5, 1.5)
            mod.weight.data.uniform_(0.5, 1.5)
            mod.bias.data.uniform_(-0.1, 0.1)
    cfg = ResNetConfig(num_channels=3, embedding_size=64, hidden_sizes=[64, 128, 256, 512], depths=[2, 2, 2, 2],
                       layer_type='basic', hidden_act='relu', downsample_in_first_stage=False)
    hf = ResNetModel(cfg).eval()
    src = ours.state_dict()

    def bn(dst, s):
        return {f'{dst}.{k}': src[f'{s}.{k}'] for k in ('weight', 'bias', 'running_mean', 'running_var')}
    m = {'embedder.embedder.convolution.weight': src['conv1.weight']}
    m.update(bn('embedder.embedder.normalization', 'bn1'))
    for li in range(4):
        for b in range(2):
            d, s = f'encoder.stages.{li}.layers.{b}', f'layer{li + 1}.{b}'
            m[f'{d}.layer.0.convolution.weight'] = src[f'{s}.conv1.weight']
            m.update(bn(f'{d}.layer.0.normalization', f'{s}.bn1'))
            m[f'{d}.layer.1.convolution.weight'] = src[f'{s}.conv2.weight']
            m.update(bn(f'{d}.layer.1.normalization', f'{s}.bn2'))
            if f'{s}.downsample.0.weight' in src:
                m[f'{d}.shortcut.convolution.weight'] = src[f'{s}.downsample.0.weight']
                m.update(bn(f'{d}.shortcut.normalization', f'{s}.downsample.1'))
    missing, unexpected = hf.load_state_dict(m, strict=False)
    assert not [k for k in missing if 'num_batches_tracked' not in k], missing
    x = torch.randn(2, 3, 96, 96)
    with torch.no_grad():
        a = ours.forward_features(x)
        b = hf(x).last_hidden_state
    assert a.shape == b.shape == (2, 512, 3, 3)
    assert (a - b).abs().max().item() <= 1e-4 * max(1.0, b.abs().max().item())


def test_slice_waveform_golden():
    from oracle.decision import slice_waveform as oslice
    from oracle.frontend import AudioConfig as OCfg
    import inference_runner as ir
    from sad.synth import synth_segment
    g = json.load(open(os.path.join(GOLDEN, 'golden_slice.json')))
    base = synth_segment(g['seed'], 0, 416000).astype(np.float32) / 32768.0
    for c in g['cases']:
        wf = base[:c['T']].copy()
        if c['silent_window']:
            amp = 32 if c['silent_window'] == 'le32' else 33
            wf[128000:256000] = np.sign(wf[128000:256000]) * amp / 32768.0
        kw = dict(sample_rate=32000, window_size=4.0, overlap=c['overlap'], silence_threshold=c.get('silence', 1e-3))
        for fn, cfg in ((oslice, OCfg(**kw)), (ir.slice_waveform, ir.AudioConfig(**kw))):
            ch, ts = fn(torch.from_numpy(wf), 32000, cfg)
            assert ts == c['timestamps'] and len(ch) == c['n']


def test_interpret_golden():
    from oracle.decision import interpret_multihead_logits as oint
    import inference_runner as ir
    for d in json.load(open(os.path.join(GOLDEN, 'golden_decide.json'))):
        t = torch.tensor(d['logits'], dtype=torch.float32)
        for fn in (oint, ir.interpret_multihead_logits):
            lab, s = fn(t, d['threshold'], d['names'], 'Real')
            assert lab == d['label']
            assert np.array_equal(s.astype(np.float32), np.array(d['probs'], dtype=np.float32))


@pytest.fixture(scope='module')
def oracle_n6():
    from oracle import resnet as ores
    return ores.load_merged_state(merged_sd('n6'))


def test_oracle_logits_match_golden(golden_frontend, golden_models, oracle_n6):
    from oracle import frontend as ofe
    imgs = ofe.resize_bilinear(torch.from_numpy(golden_frontend['std_map']).unsqueeze(1), (512, 512)).repeat(1, 3, 1, 1)
    with torch.no_grad():
        out = oracle_n6(imgs[:2])
    assert np.abs(out.numpy() - golden_models['n6_merged'][:2]).max() <= 1e-5


def test_main_json_golden(golden_frontend, golden_models):
    """Oracle aggregate + the drop-in's summarize() reproduce the reference main()'s
    JSON (plain and --smooth) from the golden per-window logits."""
    from oracle.decision import aggregate
    import inference_runner as ir
    g = json.load(open(os.path.join(GOLDEN, 'golden_main.json')))
    logits = torch.from_numpy(golden_models['n6_merged'])  # windows: pcm0, pcm1, pcm2, pcm3
    ts = [0.0, 4.0, 12.0, 16.0]
    names = [f'Synthetic{chr(65 + i)}' for i in range(6)]
    for key, smooth in (('plain', False), ('smooth', True)):
        for fn in (aggregate, ir.summarize):
            js = fn('<wav>', logits, ts, 0.5, names, 'Real', smooth, 4.0)
            assert js['segments'] == g[key]['segments']
            for k, v in g[key]['percentages'].items():
                assert abs(js['percentages'][k] - v) <= 1e-3


def test_weights_layout_matches_reference_keys():
    from oracle import resnet as ores
    from sad import weights as sw
    g = json.load(open(os.path.join(GOLDEN, 'golden_merger.json')))
    sd = sw.merged_state_dict(0, 2, False)
    keys0 = sorted(k[len('sub_models.0.'):] for k in sd if k.startswith('sub_models.0.'))
    assert keys0 == g['keys_sub0']
    ref = ores.BinaryClassifier().state_dict()
    for k, v in ref.items():
        assert tuple(sd[f'sub_models.0.{k}'].shape) == tuple(v.shape)


def test_synth_deterministic():
    from sad.synth import synth_segment
    a, b = synth_segment(0, 5), synth_segment(0, 5)
    assert np.array_equal(a, b) and a.dtype == np.int16 and a.shape == (128000,)
    assert not np.array_equal(a, synth_segment(0, 6))
    assert 2500 < a.astype(np.float64).std() < 12000 and np.abs(a).max() > 32


def test_oracle_bottleneck_resnet50_vs_transformers():
    """The Bottleneck restatement (resnet50: timm v1.5 layout, stride on the 3x3,
    1x1/s + BN downsample) equals transformers.ResNetModel(layer_type='bottleneck',
    downsample_in_bottleneck=False) given the same weights and BN statistics --
    an independent implementation pinning the oracle the deep-backbone GPU
    tests compare against (timm itself is not installed)."""
    from transformers import ResNetConfig, ResNetModel
    from oracle import resnet as ores
    torch.manual_seed(1)
    ours = ores.create_model('resnet50').eval()
    for mod in ours.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.running_mean.uniform_(-0.1, 0.1)
            mod.running_var.uniform_(0.5, 1.5)
            mod.weight.data.uniform_(0.3, 0.8)
            mod.bias.data.uniform_(-0.1, 0.1)
    cfg = ResNetConfig(num_channels=3, embedding_size=64, hidden_sizes=[256, 512, 1024, 2048], depths=[3, 4, 6, 3],
                       layer_type='bottleneck', hidden_act='relu', downsample_in_first_stage=False,
                       downsample_in_bottleneck=False)
    hf = ResNetModel(cfg).eval()
    src = ours.state_dict()

    def bn(dst, s):
        return {f'{dst}.{k}': src[f'{s}.{k}'] for k in ('weight', 'bias', 'running_mean', 'running_var')}
    m = {'embedder.embedder.convolution.weight': src['conv1.weight']}
    m.update(bn('embedder.embedder.normalization', 'bn1'))
    for li, n in enumerate((3, 4, 6, 3)):
        for b in range(n):
            d, s = f'encoder.stages.{li}.layers.{b}', f'layer{li + 1}.{b}'
            for j in range(3):
                m[f'{d}.layer.{j}.convolution.weight'] = src[f'{s}.conv{j + 1}.weight']
                m.update(bn(f'{d}.layer.{j}.normalization', f'{s}.bn{j + 1}'))
            if f'{s}.downsample.0.weight' in src:
                m[f'{d}.shortcut.convolution.weight'] = src[f'{s}.downsample.0.weight']
                m.update(bn(f'{d}.shortcut.normalization', f'{s}.downsample.1'))
    missing, unexpected = hf.load_state_dict(m, strict=False)
    assert not [k for k in missing if 'num_batches_tracked' not in k], missing
    assert not unexpected, unexpected
    x = torch.randn(2, 3, 64, 64)
    with torch.no_grad():
        a = ours.forward_features(x)
        b = hf(x).last_hidden_state
    assert a.shape == b.shape == (2, 2048, 2, 2)
    assert ((a - b).abs().max() / b.abs().max()).item() <= 1e-5


def test_segments16_recipe_matches_fixture():
    """The 16-segment recipe regenerates the PCM the reference fixture was made from."""
    import os
    import sys
    from conftest import GOLDEN
    sys.path.insert(0, GOLDEN)
    from make_golden_models16 import segments16
    pcm = segments16().astype(np.int64)
    fx = np.load(os.path.join(GOLDEN, 'golden_models16.npz'))
    assert int(pcm.sum()) == int(fx['pcm_sum'][0]) and int(np.abs(pcm).sum()) == int(fx['pcm_abs_sum'][0])
    assert fx['n6d_per_head'].shape == (16, 6, 2) and fx['n6d_merged'].shape == (16, 7)
