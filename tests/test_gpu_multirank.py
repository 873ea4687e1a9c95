"""GPU: the multi-rank branches of bench.py, bench_train.py and tools/run_1m.py, run as 2 ranks
on ONE GPU (gloo process group, --one-device; the driver's 8-GPU runs use RCCL
with one rank per GPU).  Both entry points are started with ``--gpus 2`` and no
launcher, so they must spawn the 2 ranks themselves (sad/launch.py)."""
import json
import os
import subprocess
import sys

import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _run(args, timeout=240):
    env = dict(os.environ)
    env.pop('WORLD_SIZE', None)
    r = subprocess.run([sys.executable] + args, env=env, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return r.stdout


def test_bench_two_ranks_self_launched():
    out = _run(['bench.py', '--gpus', '2', '--backend', 'gloo', '--one-device', '--batch', '64', '--steps', '2',
                '--warmup', '1', '--parity-steps', '1', '--fp32-steps', '0', '--no-cpu-baseline'])
    lines = [json.loads(s) for s in out.splitlines() if s.startswith('{')]
    assert len(lines) == 1, out
    rec = lines[0]
    assert rec['n_gpus'] == 2 and rec['config']['parallelism'] == 'dp2'
    assert len(rec['config']['per_rank_ms_per_step']) == 2 and len(rec['config']['per_rank_allgather_ms']) == 2
    assert rec['value'] > 0 and rec['parity_mode']['value'] > 0
    assert len(rec['parity_mode']['per_rank_ms_per_step']) == 2
    assert rec['parity_mode']['accuracy']['max_dlogit_golden'] <= 1e-3
    assert rec['parity_mode']['accuracy']['max_dlogit_vs_fp32_device'] <= 1e-3


def test_run_1m_two_ranks_matches_one_rank(tmp_path):
    """The 2-rank shard + all-gather returns exactly the single-rank logits
    (ragged shards: 1000 = 500 + 500 in chunks of 192, i.e. ragged chunks)."""
    sys.path.insert(0, os.path.join(ROOT, 'tools'))
    import run_1m
    common = ['--total', '1000', '--chunk', '192', '--micro-batch', '64']
    f = str(tmp_path / 'two.pt')
    _run(['tools/run_1m.py', '--gpus', '2', '--backend', 'gloo', '--one-device', '--out-logits', f] + common)
    two = torch.load(f, weights_only=True)
    rec, one = run_1m.main(common, return_logits=True)
    assert rec['gathered_rows'] == 1000 and two.shape == one.shape
    assert torch.equal(two, one)


def test_bench_train_two_ranks_self_launched():
    """bench_train.py --gpus 2 without a launcher: 2 ranks, gradient all-reduce
    over the process group, one JSON line with the whole job's segments."""
    out = _run(['bench_train.py', '--gpus', '2', '--backend', 'gloo', '--one-device', '--steps', '2', '--warmup', '1',
                '--batch-size', '4', '--pool', '16', '--eval-clips', '8'])
    lines = [json.loads(s) for s in out.splitlines() if s.startswith('{')]
    assert len(lines) == 1, out
    rec = lines[0]
    assert rec['n_gpus'] == 2 and rec['config']['parallelism'] == 'dp2'
    assert rec['segments_per_s'] > 0 and all(l == l for l in rec['train_loss_first_last'])
