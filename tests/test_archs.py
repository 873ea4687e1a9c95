"""Deeper timm ResNets -- host side, no GPU: the
deterministic state dicts carry exactly timm's keys and shapes (as restated by
the oracle), and the engine recognises the architecture from the keys."""
import pytest

from sad import weights as sw


@pytest.mark.parametrize('name', list(sw.ARCHS))
def test_state_dict_layout_matches_oracle(name):
    from oracle import resnet as ores
    ref = ores.BinaryClassifier(name).state_dict()
    mine = {f'base.{k}': v for k, v in sw.backbone_state_dict(0, name).items()}
    mine.update({f'head.{k}': v for k, v in sw.head_state_dict(1, sw.arch_spec(name)[2]).items()})
    assert list(ref.keys()) == list(mine.keys())
    for k in ref:
        assert tuple(ref[k].shape) == tuple(mine[k].shape), k
    assert sw.arch_of_state(sw.backbone_state_dict(0, name)) == name


def test_resnet18_weights_unchanged_by_generalisation():
    """resnet18's hash-seeded values depend only on its own key order."""
    a = sw.backbone_state_dict(0)
    b = sw.backbone_state_dict(0, 'resnet18')
    assert all((a[k] == b[k]).all() for k in a)


def test_unknown_arch_rejected():
    with pytest.raises(ValueError):
        sw.arch_spec('resnet26t')
    bad = sw.backbone_state_dict(0)
    bad = {k: v for k, v in bad.items() if not k.startswith('layer4.1.')}
    with pytest.raises(ValueError):
        sw.arch_of_state(bad)


def test_runner_accepts_deeper_names():
    import inference_runner as ir
    m = ir.BinaryClassifier('resnet50', init='empty')
    assert m.state_dict()['head.2.weight'].shape == (512, 2048)
    with pytest.raises(ValueError):
        ir.BinaryClassifier('vgg16', init='empty')


def test_trainer_tables_resnet34():
    from sad import train as st
    blocks = st.block_table(sw.ARCHS['resnet34'][1])
    assert [b[0] for b in blocks][:4] == ['layer1.0', 'layer1.1', 'layer1.2', 'layer2.0']
    assert sum(b[4] for b in blocks) == 3 and len(blocks) == 16
    base, head = st.init_state_dict(42, 'resnet34')
    assert list(base) == list(sw.backbone_state_dict(0, 'resnet34'))
    assert all((base[f'{b[0]}.bn2.weight'] == 0).all() for b in blocks)  # timm zero_init_last
    with pytest.raises(ValueError):
        st.init_state_dict(42, 'resnet26')


def test_trainer_tables_resnet50():
    """Bottleneck training tables: timm's key order, width / expansion, the
    downsample on every stage's first block (layer1.0 too: 64 -> 256), stride on
    conv2, zero_init_last on bn3, and the 2048-wide head input."""
    from sad import train as st
    blocks = st.bottleneck_table(sw.ARCHS['resnet50'][1])
    assert len(blocks) == 16 and [b[0] for b in blocks][:4] == ['layer1.0', 'layer1.1', 'layer1.2', 'layer2.0']
    assert blocks[0][1:] == (64, 256, 1, True, 64) and blocks[3][1:] == (256, 512, 2, True, 128)
    assert blocks[-1][1:] == (2048, 2048, 1, False, 512)
    base, head = st.init_state_dict(42, 'resnet50')
    assert list(base) == list(sw.backbone_state_dict(0, 'resnet50'))
    assert all((base[f'{b[0]}.bn3.weight'] == 0).all() for b in blocks)
    assert all((base[f'{b[0]}.bn2.weight'] == 1).all() for b in blocks)
    assert head['2.weight'].shape == (512, 2048)
    assert [n for n, _ in st.param_layout('resnet50')][-2:] == ['layer4.2.bn3.weight', 'layer4.2.bn3.bias']


def test_bench_arch_flop_counts():
    """tools/bench_arch.py's algorithmic FLOPs: resnet18 = SURVEY 8(d)'s 18.95
    GFLOP per 512x512 segment; resnet50 = timm's 4.11 GMAC at 224^2 x (512/224)^2."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tools'))
    from bench_arch import backbone_flop
    assert abs(backbone_flop('resnet18') / 1e9 - 18.95) < 0.01
    assert abs(backbone_flop('resnet50') / 2e9 / (512 / 224) ** 2 - 4.09) < 0.05
