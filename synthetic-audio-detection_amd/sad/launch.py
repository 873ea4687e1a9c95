"""One-process-per-GPU launch for the entry points that take ``--gpus N``
(bench.py, tools/run_1m.py).

When the script runs without a torch.distributed launcher (``WORLD_SIZE``
unset) and N > 1, ``relaunch`` starts ``python -m torch.distributed.run
--nproc-per-node N --master-addr 127.0.0.1`` over the same script and arguments
as a CHILD process and returns its exit code: nothing here touches the GPU, and
the parent never exec()s (the pool forbids replacing a process that
initialised the GPU; this one has not, but a child keeps the rule obvious).
Under a launcher, ``check_world`` insists that the world size is the N asked
for, so ``--gpus 8`` can never silently measure one GPU.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def under_launcher() -> bool:
    return 'WORLD_SIZE' in os.environ


def relaunch(n: int, script: str, argv: list[str]) -> int:
    """Run `script argv` as n ranks (torch.distributed.run child); its exit code."""
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={n}',
           '--master-addr=127.0.0.1', f'--master-port={free_port()}', script] + list(argv)
    env = dict(os.environ, MASTER_ADDR='127.0.0.1')
    return subprocess.run(cmd, env=env).returncode


def check_world(n_requested: int) -> tuple[int, int, int]:
    """(world, rank, local_rank) from the launcher env; raises if world != n."""
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != n_requested:
        raise SystemExit(f'--gpus {n_requested} but the launcher started {world} rank(s)')
    return world, rank, local
