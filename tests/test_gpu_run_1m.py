"""GPU: tools/run_1m.py (BASELINE configs[3] shard driver) on a small ragged
total, in process.  The host-fed mode (pinned ring of 2 chunks, double-buffered
H2D on a side stream) must produce exactly the logits of the device-synthesised
mode for the same PCM: chunks 0 and 1 are the ring's two chunks, and the ragged
chunk 2 (808 segments) replays ring chunk 0."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tools'))


def test_host_fed_matches_device_synth():
    import run_1m
    common = ['--total', '9000', '--chunk', '4096', '--micro-batch', '512']
    rec_d, dev = run_1m.main(common, return_logits=True)
    rec_h, host = run_1m.main(common + ['--host-fed'], return_logits=True)
    assert rec_d['gathered_rows'] == rec_h['gathered_rows'] == 9000
    assert rec_d['all_finite'] and rec_h['all_finite']
    assert torch.equal(host[:8192], dev[:8192])
    assert torch.equal(host[8192:], dev[:808])
