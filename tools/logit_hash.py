#!/usr/bin/env python3
"""Hash of the bench model's merged logits on the bench's synthetic batch, for
bit-identity checks of schedule switches (run it under two environments and
compare the lines):

    SAD_L2C1_SUB=0 python tools/logit_hash.py; SAD_L2C1_SUB=1 python tools/logit_hash.py
"""
import argparse
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'synthetic-audio-detection_amd')]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--dtype', default='bf16')
    ap.add_argument('--batch', type=int, default=2048)
    ap.add_argument('--micro-batch', type=int, default=1024)
    args = ap.parse_args()
    from sad import _lib
    from sad import weights as sw
    from sad.engine import Engine
    dev = torch.device('cuda:0')
    sd = sw.merged_state_dict(0, 6, False, bn_stats=sw.load_bn_stats(os.path.join(ROOT, 'tests', 'golden',
                                                                                  'bn_stats_n6.npz')))
    pcm = torch.empty(args.batch, 128000, dtype=torch.int16, device=dev)
    _lib.call('sad_synth_pcm', 0, 0, args.batch, 128000, _lib.ptr(pcm), _lib.stream_handle(dev))
    eng = Engine(sd, dev, dtype=args.dtype, micro_batch=args.micro_batch)
    _, merged = eng.forward_pcm(pcm)
    torch.cuda.synchronize()
    m = merged.cpu().contiguous()
    print(f'{args.dtype} B={args.batch} mb={args.micro_batch}: sha1 {hashlib.sha1(m.numpy().tobytes()).hexdigest()} '
          f'sum {m.double().sum().item():.9g}')


if __name__ == '__main__':
    main()
