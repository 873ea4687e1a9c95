"""GPU: the trainer's data-parallel path with two ranks (torch.distributed.run,
gloo process group, both ranks on cuda:0; the driver's 8-GPU runs use RCCL).

Each rank runs TrainNet on its own half of a 4-segment batch (per-replica BN
statistics, as DataParallel gives), all-reduces the loss, the row count and the
gradients, then clips and steps AdamW.  Checked against one process doing the
same two half-batch forwards with the global loss scale:
  * loss = the mean over the 4 rows (rel <= 1e-5), rows = 4 on both ranks;
  * clipped layer4 gradients identical on both ranks, and equal to the
    single-process sum (norm-rel <= 1e-5: same kernels, same order, except the
    all-reduce's float sum);
  * the updated layer4 weights identical on both ranks."""
import os
import subprocess
import sys

import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_two_rank_train_step_matches_single_process(tmp_path):
    env = dict(os.environ, MASTER_ADDR='127.0.0.1')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=2',
           '--master-addr=127.0.0.1', '--master-port=29533', os.path.join(ROOT, 'tests', 'ddp_train_worker.py'),
           str(tmp_path)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    o = [torch.load(tmp_path / f'rank{k}.pt', weights_only=True) for k in range(2)]
    assert o[0]['ok'] and o[1]['ok'] and o[0]['rows'] == o[1]['rows'] == 4
    assert o[0]['loss'] == o[1]['loss']
    assert torch.equal(o[0]['grad'], o[1]['grad'])
    assert torch.equal(o[0]['param'], o[1]['param'])

    # single process, same two halves, gradients summed, then the same clip
    import numpy as np
    from sad import train as st
    from sad import weights as sw
    from conftest import GOLDEN
    base = sw.backbone_state_dict(7)
    _, head = st.init_state_dict(42)
    fx = np.load(os.path.join(GOLDEN, 'golden_frontend.npz'))
    targets = torch.tensor([0, 1, 1, 0])
    net = st.TrainNet(base, head, 'cuda:0', 'fp32')
    a4, b4 = net.range4
    g_sum, loss_sum = None, 0.0
    for h in range(2):
        w = torch.from_numpy(fx['pcm'][2 * h:2 * h + 2].astype(np.float32) / 32768.0)
        img = st.TrainFrontEnd('cuda:0', 'fp32')(w.to('cuda:0'))
        feats, saved = net.forward_train(img)
        d, lc = st.ce_loss(feats, targets[2 * h:2 * h + 2], 1.0 / 4, want_grad=True)
        net.backward(d, saved)
        g = net.gflat[a4:b4].clone()
        g_sum = g if g_sum is None else g_sum + g
        loss_sum += lc[0].item()
    net.gflat[a4:b4].copy_(g_sum)
    nc = net.clip_grad_norm(a4, b4)
    torch.cuda.synchronize()
    loss = loss_sum / 4
    assert abs(o[0]['loss'] - loss) <= 1e-5 * abs(loss)
    assert abs(o[0]['norm'][0].item() - nc[0].item()) <= 1e-5 * nc[0].item()
    gref = net.gflat[a4:b4].cpu().double()
    rel = ((o[0]['grad'].double() - gref).norm() / gref.norm()).item()
    print(f'two-rank vs single-process clipped gradient: rel {rel:.2e}')
    assert rel <= 1e-5
