"""CPU: sad/launch.py -- an entry point given --gpus N without a launcher
starts N ranks itself (torch.distributed.run child, 127.0.0.1), and under a
launcher refuses a world size other than N."""
import os
import subprocess
import sys

import pytest

from conftest import PKG

WORKER = '''
import os, sys
sys.path.insert(0, {pkg!r})
import torch.distributed as dist
from sad import launch
n = int(sys.argv[1])
if n > 1 and not launch.under_launcher():
    sys.exit(launch.relaunch(n, os.path.abspath(__file__), sys.argv[1:]))
world, rank, local = launch.check_world(n)
dist.init_process_group('gloo')
import torch
t = torch.tensor([rank + 1.0])
dist.all_reduce(t)
print(f'rank {{rank}} world {{world}} sum {{t.item():.0f}}', flush=True)
dist.destroy_process_group()
'''


def test_relaunch_two_ranks(tmp_path):
    script = tmp_path / 'w.py'
    script.write_text(WORKER.format(pkg=PKG))
    env = dict(os.environ)
    env.pop('WORLD_SIZE', None)
    r = subprocess.run([sys.executable, str(script), '2'], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert 'rank 0 world 2 sum 3' in r.stdout and 'rank 1 world 2 sum 3' in r.stdout


def test_world_mismatch_refused(monkeypatch):
    from sad import launch
    monkeypatch.setenv('WORLD_SIZE', '1')
    with pytest.raises(SystemExit):
        launch.check_world(8)
    monkeypatch.setenv('WORLD_SIZE', '8')
    monkeypatch.setenv('RANK', '3')
    monkeypatch.setenv('LOCAL_RANK', '3')
    assert launch.check_world(8) == (8, 3, 3)
