"""CPU (gloo, world_size 2 and 3): segment sharding and the logit all-gather
used by multi-GPU inference (sad.distributed), incl. ragged shards."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from sad.distributed import gather_rows, shard_range


def test_shard_range_covers_exactly():
    for n in (0, 1, 7, 2048, 1000001):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    s, e = shard_range(n, rank, world)
    # each rank "computes" logits for its segments: row i = [i, i+0.5, ...]
    local = torch.arange(s, e, dtype=torch.float32)[:, None] + torch.tensor([0.0, 0.5, 0.25])
    full = gather_rows(local, n)
    q.put((rank, full.numpy().tolist()))
    dist.destroy_process_group()


def _run(world, n):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    ref = (torch.arange(n, dtype=torch.float32)[:, None] + torch.tensor([0.0, 0.5, 0.25])).tolist()
    for _, full in res:
        assert full == ref


def test_gather_rows_world2_ragged():
    _run(2, 7)


def test_gather_rows_world3():
    _run(3, 10)


def _trainer_worker(rank, world, port, q):
    """submodel_trainer's cross-rank reductions (validation totals, prediction
    gathering) on a gloo group: rank r contributes loss r+1, r correct of r+2."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import submodel_trainer as smt

    class _T:
        device = 'cpu'
    model = smt.DeviceModel(_T(), None, rank, world, dist.group.WORLD)
    tot = smt._allreduce_sum([float(rank + 1), float(rank), float(rank + 2)], model)
    preds, tgts = smt._gather_lists([rank] * (rank + 1), [10 + rank] * (rank + 1), model)
    q.put((rank, tot, preds, tgts))
    dist.destroy_process_group()


def test_trainer_reductions_world2():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_trainer_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for rank, tot, preds, tgts in res:
        assert tot == [3.0, 1.0, 5.0]
        assert preds == [0, 1, 1] and tgts == [10, 11, 11]
