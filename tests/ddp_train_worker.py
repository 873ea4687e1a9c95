"""Worker for tests/test_gpu_train_ddp.py (not a test module): one rank of a
2-rank data-parallel trainer step (torch.distributed.run, gloo process group,
both ranks on cuda:0).  Rank r trains on segments [2r, 2r+2) of the golden PCM
and writes its loss, clipped layer4 gradients and updated layer4 weights to
<out_dir>/rank<r>.pt."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'synthetic-audio-detection_amd')]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    out_dir = sys.argv[1]
    dist.init_process_group('gloo')
    rank, world = dist.get_rank(), dist.get_world_size()
    from sad import train as st
    from sad import weights as sw
    base = sw.backbone_state_dict(7)
    _, head = st.init_state_dict(42)
    fx = np.load(os.path.join(ROOT, 'tests', 'golden', 'golden_frontend.npz'))
    w = torch.from_numpy(fx['pcm'][2 * rank:2 * rank + 2].astype(np.float32) / 32768.0)
    targets = torch.tensor([0, 1, 1, 0])[2 * rank:2 * rank + 2]
    dev = torch.device('cuda', 0)
    img = st.TrainFrontEnd(dev, 'fp32')(w.to(dev))
    tr = st.Trainer(base, head, dev, 'fp32', group=dist.group.WORLD, world=world)
    loss, correct, rows, ok = tr.train_step(img, targets)  # global batch from the all-reduce
    torch.cuda.synchronize()
    a4, b4 = tr.net.range4
    torch.save({'loss': loss, 'rows': rows, 'ok': ok, 'norm': tr.last_norm.cpu(),
                'grad': tr.net.gflat[a4:b4].cpu(), 'param': tr.net.pflat[a4:b4].cpu()},
               os.path.join(out_dir, f'rank{rank}.pt'))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
