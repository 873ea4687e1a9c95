"""CPU: host-side validation in sad/engine.py before raw pointers reach the C
plan builders (shapes against the timm layout; unknown Bottleneck depths
refused instead of being read as resnet18), and the split-bf16 layout helpers."""
import pytest
import torch


def test_backbone_shape_mismatch_raises():
    from sad import weights as sw
    from sad.engine import _backbone_arrays
    sd = sw.backbone_state_dict(0, 'resnet18')
    assert len(_backbone_arrays(sd, sw.arch_param_shapes('resnet18'))) == 100
    bad = dict(sd)
    bad['layer1.0.conv1.weight'] = torch.zeros(128, 64, 3, 3)  # a wider net
    with pytest.raises(ValueError, match='layer1.0.conv1.weight'):
        _backbone_arrays(bad, sw.arch_param_shapes('resnet18'))
    del bad['layer1.0.conv1.weight']
    with pytest.raises(KeyError):
        _backbone_arrays(bad, sw.arch_param_shapes('resnet18'))


def test_unknown_bottleneck_depth_refused():
    from sad import weights as sw
    from sad.engine import _arch
    sd = sw.backbone_state_dict(0, 'resnet50')
    assert _arch(sd) == 'resnet50'
    # drop layer3 blocks 2..5: a (3, 4, 2, 3) Bottleneck net matches no timm name
    cut = {k: v for k, v in sd.items() if not any(k.startswith(f'layer3.{b}.') for b in range(2, 6))}
    with pytest.raises(ValueError):
        _arch(cut)
    # a BasicBlock key set with a missing block still maps to resnet18 (missing-key check names it)
    sd18 = sw.backbone_state_dict(0, 'resnet18')
    assert _arch({k: v for k, v in sd18.items() if not k.startswith('layer4.1.')}) == 'resnet18'


def test_head_shape_checked_against_feature_width():
    from sad import weights as sw
    from sad.engine import _head_arrays
    head = sw.head_state_dict(0, 512)
    assert len(_head_arrays(head, 512)) == 14
    with pytest.raises(ValueError, match='2.weight'):
        _head_arrays(head, 2048)  # a resnet50 backbone (2048 features) with a 512-input head


def test_split_layout_roundtrip():
    from sad.engine import from_split, to_split
    x = torch.randn(3, 5, 96, dtype=torch.float32) * 7
    s = to_split(x)
    assert s.dtype == torch.bfloat16 and s.shape == (3, 5, 192)
    # hi in the first 32 of each 64, lo in the next 32
    assert torch.equal(s[..., :32].float(), x[..., :32].to(torch.bfloat16).float())
    back = from_split(s)
    rel = ((back - x).abs() / x.abs().clamp_min(1e-30)).max().item()
    assert rel <= 2.0 ** -16, rel
