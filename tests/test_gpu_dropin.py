"""GPU: the drop-in modules end to end.

* inference_runner.main on the fixture WAV reproduces the JSON that the
  REFERENCE's main() wrote for the same file and checkpoint
  (tests/golden/golden_main.json): identical segments/labels/timestamps,
  percentages within 1e-3 (they are 100 x mean sigmoid).
* the reference-shaped model call model(x[B,3,512,512]) equals the fused
  map path; waveform_to_spectrogram matches the oracle.
* sad_conv2d_run (one BasicBlock conv) matches torch conv2d (+bias, residual,
  ReLU) in fp32, incl. stride 2, 1x1 shortcut and a ragged M tail.
"""
import json
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import GOLDEN, merged_sd

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'


@pytest.fixture(scope='module')
def merged_path(tmp_path_factory):
    p = tmp_path_factory.mktemp('m') / 'merged_n6.pth'
    names = [f'Synthetic{chr(65 + i)}' for i in range(6)] + ['Real']
    torch.save({'state_dict': merged_sd('n6'), 'metadata': {'class_names': names}}, p)
    return str(p)


def _fixture_wav(path, golden_frontend):
    from sad.audio import save_pcm16
    from sad.synth import synth_segment
    pcm = golden_frontend['pcm']
    silent = (synth_segment(5, 0) // 2048).astype(np.int16)
    wav = np.concatenate([pcm[0], pcm[1], silent, pcm[2], pcm[3], pcm[0][:77777]])
    save_pcm16(path, wav)


@pytest.mark.parametrize('smooth', [False, True])
def test_inference_runner_main_matches_reference_json(tmp_path, merged_path, golden_frontend, smooth):
    import inference_runner as ir
    g = json.load(open(os.path.join(GOLDEN, 'golden_main.json')))['smooth' if smooth else 'plain']
    wav = str(tmp_path / 'clip.wav')
    _fixture_wav(wav, golden_frontend)
    out = str(tmp_path / 'out.json')
    js = ir.main(['--merged-model', merged_path, '--audio', wav, '--output-json', out] + (['--smooth'] if smooth else []))
    on_disk = json.load(open(out))
    assert on_disk['segments'] == g['segments'] == js['segments']
    assert set(on_disk['percentages']) == set(g['percentages'])
    for k, v in g['percentages'].items():
        assert abs(on_disk['percentages'][k] - v) <= 1e-3, (k, on_disk['percentages'][k], v)
    assert on_disk['filename'] == wav


def test_empty_audio_json(tmp_path, merged_path):
    import inference_runner as ir
    from sad.audio import save_pcm16
    wav = str(tmp_path / 'quiet.wav')
    save_pcm16(wav, np.zeros(200000, np.int16))
    out = str(tmp_path / 'o.json')
    ir.main(['--merged-model', merged_path, '--audio', wav, '--output-json', out])
    assert json.load(open(out)) == {'filename': wav, 'segments': [], 'percentages': {}}


def test_missing_metadata_raises(tmp_path):
    import inference_runner as ir
    p = tmp_path / 'bad.pth'
    torch.save({'state_dict': {}}, p)
    with pytest.raises(ValueError, match='metadata'):
        ir.load_merged_model(str(p), torch.device(DEV))


def test_image_path_equals_map_path(merged_path, golden_frontend):
    import inference_runner as ir
    model, _ = ir.load_merged_model(merged_path, torch.device(DEV))
    spec_cfg = ir.SpectrogramConfig()
    wf = torch.from_numpy(golden_frontend['pcm'][1].astype(np.float32) / 32768.0)
    img = ir.waveform_to_spectrogram(wf, 32000, spec_cfg)
    assert img.shape == (1, 3, 512, 512)
    from oracle import frontend as ofe
    ref = ofe.waveform_to_spectrogram(wf, 32000, ofe.SpectrogramConfig())
    assert (img.cpu() - ref).abs().max().item() <= 2e-4
    a = model(img)
    b = model.forward_maps(torch.from_numpy(golden_frontend['std_map'][1:2]))
    assert (a - b).abs().max().item() <= 5e-4
    # distinct channels run the 3-channel stem (parity: test_gpu_img3.py)
    c = model(torch.randn(1, 3, 512, 512))
    assert c.shape == a.shape and torch.isfinite(c).all()


@pytest.mark.parametrize('N,H,Cin,Cout,k,s,p,res', [
    (3, 20, 64, 64, 3, 1, 1, True),      # ragged M (1200 rows), residual
    (2, 17, 64, 128, 3, 2, 1, False),    # stride 2, odd size
    (2, 16, 128, 256, 1, 2, 0, False),   # 1x1 shortcut
    (1, 8, 512, 512, 3, 1, 1, True),     # deep K
])
def test_conv_op_fp32_vs_torch(N, H, Cin, Cout, k, s, p, res):
    from sad.engine import conv2d
    torch.manual_seed(0)
    x = torch.randn(N, H, H, Cin, device=DEV)
    w = torch.randn(Cout, k, k, Cin, device=DEV) * (2.0 / (k * k * Cin)) ** 0.5
    b = torch.randn(Cout, device=DEV)
    Ho = (H + 2 * p - k) // s + 1
    r = torch.randn(N, Ho, Ho, Cout, device=DEV) if res else None
    for v in (0, 1, 5):
        if Cout % 128 and v == 5:
            continue
        y = conv2d(x, w, b, s, p, r, True, v)
        ref = F.conv2d(x.permute(0, 3, 1, 2).double(), w.permute(0, 3, 1, 2).double(), b.double(), s, p)
        ref = ref.permute(0, 2, 3, 1)
        if res:
            ref = ref + r.double()
        ref = ref.clamp_min(0).float()
        err = (y - ref).abs().max().item() / ref.abs().max().item()
        assert err <= 1e-5, (v, err)


@pytest.mark.parametrize('N,H,Cin,Cout,stride,shortcut', [
    (3, 20, 64, 64, 1, 'identity'),     # layer1-style block conv2 + identity, ragged M
    (2, 18, 64, 128, 2, None),          # block conv1 with stride 2
    (2, 16, 128, 128, 1, 'ds'),         # conv2 + downsample shortcut from a 32x32 input
    (1, 8, 512, 512, 1, 'identity'),    # deep K
    (2, 16, 64, 64, 1, 'identity'),     # halo (16x16 tiles), layer1-style, one tile per image
    (3, 48, 64, 64, 1, None),           # halo, plain conv1, 9 tiles per image, fewer tiles than CUs
    (16, 128, 64, 64, 1, 'identity'),   # halo at layer1's map size, several tiles per workgroup
    (2, 32, 128, 64, 1, 'identity'),    # halo, two 64-channel chunks per tile
    (2, 32, 128, 128, 1, 'ds'),         # downsample shortcut from 64x64
    (1, 16, 512, 512, 1, 'identity'),   # deep K, Cout 512
])
def test_block_conv_fp32_vs_torch(N, H, Cin, Cout, stride, shortcut):
    """conv + shortcut as one GEMM == torch conv2d + (identity | 1x1/2 conv) + bias, ReLU."""
    from sad.engine import block_conv
    torch.manual_seed(0)
    x = torch.randn(N, H, H, Cin, device=DEV)
    w = torch.randn(Cout, 3, 3, Cin, device=DEV) * (2.0 / (9 * Cin)) ** 0.5
    b = torch.randn(Cout, device=DEV)
    Ho = (H + 2 - 3) // stride + 1
    ref = F.conv2d(x.permute(0, 3, 1, 2).double(), w.permute(0, 3, 1, 2).double(), b.double(), stride, 1)
    if shortcut == 'identity':
        sc = torch.randn(N, Ho, Ho, Cout, device=DEV)
        wsc = torch.eye(Cout, device=DEV)
        ref = ref + sc.permute(0, 3, 1, 2).double()
        ss = 1
    elif shortcut == 'ds':
        Cs = 64
        sc = torch.randn(N, 2 * Ho, 2 * Ho, Cs, device=DEV)
        wsc = torch.randn(Cout, Cs, device=DEV) * 0.1
        ref = ref + F.conv2d(sc.permute(0, 3, 1, 2).double(), wsc.double()[:, :, None, None], None, 2)
        ss = 2
    else:
        sc, wsc, ss = None, None, 1
    wcat = w.reshape(Cout, -1) if sc is None else torch.cat([w.reshape(Cout, -1), wsc], 1)
    ref = ref.permute(0, 2, 3, 1).clamp_min(0).float()
    bc = {9: 64, 10: 128, 11: 64, 12: 128, 13: 256, 14: 128, 15: 128, 16: 64, 17: 256, 18: 128}
    vs = [0] + [v for v in bc if Cout % bc[v] == 0]
    for v in vs:
        y = block_conv(x, wcat.contiguous(), b, stride, 1, sc, ss, True, v)
        err = (y - ref).abs().max().item() / ref.abs().max().item()
        assert err <= 1e-5, (v, err)
    # bf16: default kernel choice (the halo kernel for Cout 64 without a GEMM shortcut)
    wb = wcat.contiguous().bfloat16()
    yb = block_conv(x.bfloat16(), wb, b, stride, 1, None if sc is None else sc.bfloat16(), ss, True)
    assert (yb.float() - ref).abs().max().item() / ref.abs().max().item() <= 3e-2
    if stride == 1 and H % 16 == 0 and shortcut != 'ds':
        # halo kernel, identity shortcut as an epilogue residual; the weight rows keep
        # their (unused) identity columns, as the backbone plan stores them
        res = None if sc is None else sc.bfloat16()
        yh = block_conv(x.bfloat16(), wb, b, 1, 1, None, 1, True, 20, res=res)
        assert (yh.float() - ref).abs().max().item() / ref.abs().max().item() <= 3e-2
        # same bf16 operands through the implicit-GEMM kernel: the two agree to bf16 rounding
        yg = block_conv(x.bfloat16(), wb, b, 1, 1, res, 1, True, 9)
        assert (yh.float() - yg.float()).abs().max().item() / yg.float().abs().max().item() <= 1e-2
