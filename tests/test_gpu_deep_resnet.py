"""GPU parity of the deeper timm ResNets (resnet34 BasicBlocks, resnet50
Bottlenecks) on libsad's generic ResNet plan against the
CPU oracle, end to end from the golden maps to the merged logits.

The hash-seeded weights get BN running statistics calibrated on the test maps
themselves (oracle in train mode, cumulative averages), so activations stay
O(1) through 16-33 blocks.  Tolerances: fp32 and split-bf16 (bf16x3) modes
|dlogit| <= 1e-3 (the north-star bar); bf16 mode pooled features relative error <= 5e-2 / 1e-1 / 2e-1
for resnet34 / 50 / 101 (reported, not the parity gate).  parity pinned only through the oracle (no reference
fixture exists for these backbones)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = 'cuda:0'


def _calibrated(name, maps):
    from oracle import frontend as ofe
    from oracle import resnet as ores
    from sad import weights as sw
    sd = sw.merged_state_dict(0, 2, False, model_name=name)
    model = ores.load_merged_state(sd, name)
    img = ofe.resize_bilinear(maps.unsqueeze(1), (512, 512)).repeat(1, 3, 1, 1)
    for m in model.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.reset_running_stats()
            m.momentum = None
    model.train()
    with torch.no_grad():
        model.sub_models[0].base.forward_features(img)
        for sm in model.sub_models[1:]:
            sm.base.load_state_dict(model.sub_models[0].base.state_dict())
    model.eval()
    with torch.no_grad():
        ref = model(img)
        feats = model.sub_models[0].base(img)
    return model.state_dict(), ref, feats


@pytest.fixture(scope='module')
def maps(golden_frontend):
    return torch.from_numpy(golden_frontend['std_map'][:3]).contiguous()


@pytest.mark.parametrize('name', ['resnet50', 'resnet34', 'resnet101'])
def test_deep_resnet_vs_oracle(name, maps):
    from sad.engine import Engine, ResNetBackbone
    sd, ref, ref_feats = _calibrated(name, maps)
    eng = Engine(sd, DEV, dtype='fp32', micro_batch=2)  # ragged tail: 3 = 2 + 1
    assert eng.arch == name and len(eng.backbones) == 1 and isinstance(eng.backbones[0], ResNetBackbone)
    _, merged = eng.forward_maps(maps.to(DEV))
    feats = eng.backbones[0](maps.to(DEV))
    torch.cuda.synchronize()
    df = ((feats.cpu() - ref_feats).abs().max() / ref_feats.abs().max()).item()
    d = (merged.cpu() - ref).abs().max().item()
    print(f'{name} fp32: pooled rel err {df:.3e}, max|dlogit| {d:.3e}')
    assert np.isfinite(merged.cpu().numpy()).all()
    assert d <= 1e-3

    # the split-bf16 parity mode: four products in the Bottleneck plans
    eng3 = Engine(sd, DEV, dtype='bf16x3', micro_batch=2)
    _, merged3 = eng3.forward_maps(maps.to(DEV))
    torch.cuda.synchronize()
    d3 = (merged3.cpu() - ref).abs().max().item()
    print(f'{name} bf16x3: max|dlogit| {d3:.3e}')
    assert d3 <= 1e-3

    eng16 = Engine(sd, DEV, dtype='bf16', micro_batch=3)
    f16 = eng16.backbones[0](maps.to(DEV))
    torch.cuda.synchronize()
    e16 = ((f16.cpu() - ref_feats).abs().max() / ref_feats.abs().max()).item()
    print(f'{name} bf16: pooled rel err {e16:.3e}')
    # bf16 noise grows with depth (resnet50: the CPU emulation of the bf16
    # arithmetic is itself 6.9e-2 off, test_resnet50_bf16_vs_emulated_oracle)
    assert e16 <= {'resnet34': 5e-2, 'resnet50': 1e-1, 'resnet101': 2e-1}[name]


def test_deep_resnet_image_entry_matches_map_entry(maps):
    """sad_resnet_run_img on the resized image == sad_resnet_run on the map."""
    from sad.engine import ResNetBackbone, resize
    from sad import weights as sw
    base = sw.backbone_state_dict(0, 'resnet50')
    bb = ResNetBackbone(base, 'resnet50', DEV, 'fp32', micro_batch=3)
    m = maps.to(DEV)
    a = bb(m)
    b = bb.forward_images(resize(m))
    torch.cuda.synchronize()
    err = ((a - b).abs().max() / a.abs().max()).item()
    assert err <= 1e-5, err


def test_merger_and_runner_cli_resnet50(tmp_path, golden_frontend):
    """model_merger.main --model-name resnet50 -> inference_runner.main
    --model-name resnet50 on a 4-window WAV; the JSON equals summarize() of the
    oracle's merged logits (same segments/labels, percentages within 1e-3)."""
    import csv
    import json

    import inference_runner as ir
    import model_merger as mm
    from oracle import frontend as ofe
    from sad.audio import save_pcm16
    pcm = golden_frontend['pcm'][:4]
    _, maps = ofe.batch_maps(pcm)
    sd, ref, _ = _calibrated('resnet50', maps)
    rows = []
    for i in range(2):
        sub = {k[len(f'sub_models.{i}.'):]: v for k, v in sd.items() if k.startswith(f'sub_models.{i}.')}
        torch.save({'state_dict': sub}, tmp_path / f'sub{i}.pth')
        rows.append({'model_filename': f'sub{i}.pth', 'synthetic_class': f'Syn{i}', 'real_class': 'Real'})
    with open(tmp_path / 'm.csv', 'w', newline='') as f:
        w = csv.DictWriter(f, fieldnames=['model_filename', 'synthetic_class', 'real_class'])
        w.writeheader()
        w.writerows(rows)
    merged = str(tmp_path / 'merged.pth')
    names = mm.main(['--submodels-folder', str(tmp_path), '--csv-file', str(tmp_path / 'm.csv'),
                     '--model-name', 'resnet50', '--output-path', merged])
    assert names == ['Syn0', 'Syn1', 'Real']
    wav = str(tmp_path / 'clip.wav')
    save_pcm16(wav, np.concatenate(list(pcm)))
    out = str(tmp_path / 'o.json')
    js = ir.main(['--merged-model', merged, '--audio', wav, '--output-json', out, '--model-name', 'resnet50'])
    exp = ir.summarize(wav, list(ref), [0.0, 4.0, 8.0, 12.0], 0.5, ['Syn0', 'Syn1'], 'Real', False, 4.0)
    assert js['segments'] == exp['segments']
    for k, v in exp['percentages'].items():
        assert abs(js['percentages'][k] - v) <= 1e-3, (k, js['percentages'][k], v)


def _bf(x):
    return x.to(torch.bfloat16).float()


def _emulated_bf16_features(model, img):
    """The bf16 plan's arithmetic on the CPU: BN folded into each conv in
    float64, weights rounded once to bf16, activations rounded to bf16 after
    every conv (+ shortcut) + ReLU, fp32 accumulation; the stem sums the 3
    identical input channels (resnet.hip / api.hip fold_stem)."""
    import torch.nn.functional as F

    def fold(conv, bn):
        s = bn.weight.double() / torch.sqrt(bn.running_var.double() + 1e-5)
        w = _bf((conv.weight.double() * s.view(-1, 1, 1, 1)).float())
        b = (bn.bias.double() - bn.running_mean.double() * s).float()
        return w, b

    base = model.base
    w, b = fold(base.conv1, base.bn1)
    x = F.conv2d(_bf(img[:, :1]), w.sum(1, keepdim=True), b, stride=2, padding=3)
    x = _bf(F.max_pool2d(F.relu(x), 3, 2, 1))
    for li in range(1, 5):
        for blk in getattr(base, f'layer{li}'):
            w1, b1 = fold(blk.conv1, blk.bn1)
            w2, b2 = fold(blk.conv2, blk.bn2)
            w3, b3 = fold(blk.conv3, blk.bn3)
            t = _bf(F.relu(F.conv2d(x, w1, b1)))
            t = _bf(F.relu(F.conv2d(t, w2, b2, stride=blk.conv2.stride, padding=1)))
            y = F.conv2d(t, w3, b3)
            if blk.downsample is not None:
                wd, bd = fold(blk.downsample[0], blk.downsample[1])
                y = y + F.conv2d(x, wd, bd, stride=blk.downsample[0].stride)
            else:
                y = y + x
            x = _bf(F.relu(y))
    return x.mean(dim=(2, 3))


def test_resnet50_bf16_vs_emulated_oracle(maps):
    """bf16 mode against the same arithmetic emulated on the CPU.  Measured:
    the emulation itself sits 6.9e-2 (relative, pooled features) from the fp32
    oracle and the GPU 8.0e-2 from the emulation -- bf16 rounding flips from a
    different fp32 summation order grow through the 16 Bottlenecks as much as
    the bf16 rounding itself, so the bar is "same order as the inherent bf16
    noise" (a wrong weight layout or tap order gives O(1) errors)."""
    from oracle import frontend as ofe
    from sad.engine import Engine
    sd, _, ref_fp32 = _calibrated('resnet50', maps)
    from oracle import resnet as ores
    model = ores.load_merged_state(sd, 'resnet50')
    img = ofe.resize_bilinear(maps.unsqueeze(1), (512, 512)).repeat(1, 3, 1, 1)
    with torch.no_grad():
        emu = _emulated_bf16_features(model.sub_models[0], img)
    eng = Engine(sd, DEV, dtype='bf16', micro_batch=3)
    f16 = eng.backbones[0](maps.to(DEV))
    torch.cuda.synchronize()
    e_emu = ((f16.cpu() - emu).abs().max() / emu.abs().max()).item()
    e_emu_fp32 = ((emu - ref_fp32).abs().max() / ref_fp32.abs().max()).item()
    print(f'resnet50 bf16 vs emulated {e_emu:.3e}; emulated vs fp32 oracle {e_emu_fp32:.3e}')
    assert e_emu <= max(2.5 * e_emu_fp32, 2e-2)
