#!/usr/bin/env python3
"""Training benchmark (BASELINE.json configs[4]): submodel_trainer.py's
data-parallel step -- device front end (mel norm=None, SpecAugment,
RandomResizedCrop) + train-mode ResNet-18 forward + CE on pooled features +
layer4 backward + RCCL all-reduce of the gradients + clip + AdamW -- on 1..8
MI355X, one process per GPU: under torchrun, or started bare with --gpus N,
in which case it starts the N ranks itself (sad/launch.py, like bench.py).

``--head-loss`` trains through model.head (submodel_trainer.py --head-loss):
CE and both accuracies on the BinaryClassifier's two logits; by default they
run on the 512 pooled features as in the reference (quirk C1), where the
eval accuracy of a two-class problem says little.

Workload per rank and step: ``--batch-size`` files (default 32, the reference
default) x 2 segments = 64 segments of synthetic labelled audio
(sad.synth.synth_labelled_clip: class 1 = noise + harmonic stack, class 0 =
low-passed noise), resident in HBM.  Prints one JSON line on rank 0: steps/s,
segments/s (whole job), train accuracy over the timed steps, and the eval-mode
accuracy on held-out clips after training.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'synthetic-audio-detection_amd')]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FWD_FLOP = 18.13e9   # per segment (bench.py / DESIGN.md section 4)
BWD_FLOP = 8.6e9     # layer4 dgrad + wgrad per segment


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--batch-size', type=int, default=32, help='files per GPU per step (2 segments each)')
    ap.add_argument('--dtype', default='bf16', choices=['bf16', 'mixed', 'fp32'])
    ap.add_argument('--pool', type=int, default=256, help='synthetic training clips per rank')
    ap.add_argument('--eval-clips', type=int, default=64)
    ap.add_argument('--lr', type=float, default=1e-3)
    ap.add_argument('--head-loss', action='store_true',
                    help="submodel_trainer.py --head-loss: CE / accuracy on model.head's 2 logits (default: the "
                         "reference's pooled features, quirk C1)")
    ap.add_argument('--backend', default='nccl', choices=['nccl', 'gloo'], help='gloo: tests only')
    ap.add_argument('--one-device', action='store_true', help='every rank on cuda:0 (2-rank test on one GPU)')
    args = ap.parse_args()
    from sad import launch
    if args.gpus > 1 and not launch.under_launcher():
        # started bare with --gpus N: N ranks as a torch.distributed.run child (sad/launch.py)
        sys.exit(launch.relaunch(args.gpus, os.path.abspath(__file__), sys.argv[1:]))
    world, rank, local = launch.check_world(args.gpus)
    dev = torch.device('cuda', 0 if args.one_device else local)
    torch.cuda.set_device(dev)
    group = None
    if world > 1:
        if args.backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
        else:
            dist.init_process_group('gloo')
        group = dist.group.WORLD

    from sad import augment
    from sad import train as st
    from sad.synth import synth_labelled_clip
    torch.manual_seed(42)
    base, head = st.init_state_dict(42)
    tr = st.Trainer(base, head, dev, args.dtype, lr=args.lr, group=group, world=world, head_loss=args.head_loss)
    fe = st.TrainFrontEnd(dev, args.dtype)
    P = args.pool
    labels = np.arange(P) % 2
    clips = np.stack([synth_labelled_clip(rank, i, int(labels[i])) for i in range(P)])
    wav = torch.from_numpy(clips.astype(np.float32) / 32768.0).to(dev)        # [P, 256000]
    lab = torch.from_numpy(labels).long()
    g = torch.Generator().manual_seed(1000 + rank)
    B = args.batch_size

    def make_batch():
        # what the DataLoader workers hand over: file indices and the augmentation
        # parameters they drew (host RNG, off the critical path in the trainer)
        idx = torch.randint(0, P, (B,), generator=g)
        masks = torch.tensor([augment.specaug_masks(generator=g) for _ in range(2 * B)], dtype=torch.int32)
        boxes = torch.tensor([augment.random_resized_crop_params(generator=g) for _ in range(2 * B)],
                             dtype=torch.int32)
        return idx.to(dev), torch.cat([lab[idx], lab[idx]]).to(dev), masks.to(dev), boxes.to(dev)

    batches = [make_batch() for _ in range(args.warmup + args.steps)]
    it = iter(batches)

    def step():
        idx, t, masks, boxes = next(it)
        waves = torch.cat([wav[idx, :128000], wav[idx, 128000:]], dim=0)
        img = fe(waves, masks, boxes)
        # every rank takes 2 x batch-size segments: the global batch is known, so
        # the step needs no all-reduce + host read of it
        return tr.train_step(img, t, global_batch=img.shape[0] * world)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    correct = rows = 0
    losses = []
    for _ in range(args.steps):
        loss, c, n, ok = step()
        correct += c
        rows += n
        losses.append(loss)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    # eval-mode accuracy on held-out clips (BN folded with the running stats)
    bb = tr.net.eval_backbone()
    E = args.eval_clips
    el = np.arange(E) % 2
    ev = torch.from_numpy(np.stack([synth_labelled_clip(10_000 + rank, i, int(el[i]))[:128000]
                                    for i in range(E)]).astype(np.float32) / 32768.0).to(dev)
    feats = bb(fe.maps(ev))
    if args.head_loss:
        feats = tr.net.head_forward(feats, train=False)
    _, lc = st.ce_loss(feats, torch.from_numpy(el).long())
    eval_correct = lc[1].item()
    if world > 1:
        t = torch.tensor([eval_correct, float(E)], device=dev)
        dist.all_reduce(t)
        eval_correct, E = t.tolist()
    seg_s = rows / elapsed
    if rank == 0:
        achieved = (FWD_FLOP + BWD_FLOP) * seg_s / world / 1e12
        print(json.dumps({
            'metric': 'submodel_trainer data-parallel training steps/sec (bf16, RCCL all-reduce)',
            'value': round(args.steps / elapsed, 3), 'unit': 'steps/s', 'segments_per_s': round(seg_s, 1),
            'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': round(elapsed * 1e3 / args.steps, 3), 'higher_is_better': True, 'scaling': 'weak',
            'dtype': args.dtype, 'data': 'synthetic labelled clips (noise+harmonics vs low-passed noise), HBM-resident',
            'config': {'workload': 'train step: front end + train-mode ResNet-18 fwd + CE + layer4 bwd + '
                                   'all-reduce + clip + AdamW', 'files_per_gpu': B, 'segments_per_gpu': 2 * B,
                       'parallelism': f'dp{world}'},
            'head_loss': args.head_loss,
            'train_loss_first_last': [round(losses[0], 4), round(losses[-1], 4)],
            'train_accuracy_timed_steps': round(100.0 * correct / max(rows, 1), 2),
            'eval_accuracy_after': round(100.0 * eval_correct / E, 2),
            'roofline': {'bound': 'mfma', 'achieved': round(achieved, 1), 'peak': 2500.0, 'unit': 'TFLOP/s',
                         'frac': round(achieved / 2500.0, 4), 'flop_per_segment': FWD_FLOP + BWD_FLOP},
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
