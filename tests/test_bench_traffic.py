"""bench.py's roofline.traffic: the dominant kernel's PMC record must resolve in
the committed traffic file (a hard-coded template key went
stale and the driver's line carried traffic = null)."""
import json
import os

import pytest

import bench


def test_traffic_file_committed():
    tf = bench.traffic_file('bf16')
    assert tf and os.path.exists(tf)


@pytest.mark.parametrize('dtype', ['bf16', 'bf16x3'])
def test_dominant_kernel_resolves_in_committed_traffic(dtype):
    tf = bench.traffic_file(dtype)
    if dtype == 'bf16x3' and not tf:
        pytest.skip('no committed split-bf16 PMC traffic file yet')
    with open(tf) as f:
        tr = json.load(f)
    prefix = bench.DOMINANT[dtype][1]
    keys = [k for k in tr if k.startswith(prefix)]
    assert keys, f'no {prefix}* record in {tf}'
    t = bench.dominant_traffic(tr, prefix)
    assert t is not None and t > 0
    # per-launch memory-side bytes of a 1,024-segment layer3/4 conv: between
    # the output map alone and 4x the algorithmic operand bytes
    assert 2e8 < t < 6e9


def test_dominant_traffic_weights_by_launches():
    tr = {'k<1>|1': {'launches_per_step': 3, 'hbm_read_bytes': 100.0, 'hbm_write_bytes': 0.0},
          'k<2>|1': {'launches_per_step': 1, 'hbm_read_bytes': 500.0, 'hbm_write_bytes': 100.0},
          'other|1': {'launches_per_step': 9, 'hbm_read_bytes': 1e9, 'hbm_write_bytes': 1e9}}
    assert bench.dominant_traffic(tr, 'k<') == round((3 * 100 + 600) / 4)
    assert bench.dominant_traffic(tr, 'missing<') is None
    tr['k<3>|1'] = {'launches_per_step': 1, 'hbm_read_bytes': None, 'hbm_write_bytes': None}
    assert bench.dominant_traffic(tr, 'k<') is None
