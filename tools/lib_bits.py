"""A/B helper (GPU box): the front end's dB + standardised maps, the stem and
the merged logits of one library build (SAD_LIB) on a fixed synthetic batch,
saved to an .npz as SHA-256 digests plus the first 2 segments (the files stay
small) -- two builds' files are then compared bit for bit.
    SAD_LIB=tools/_libsad_base.so python tools/lib_bits.py out_base.npz"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'synthetic-audio-detection_amd'), os.path.join(ROOT, 'tests')]

import hashlib  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from conftest import merged_sd
    from sad import _lib
    from sad.engine import Engine
    dev = torch.device('cuda:0')
    B = 512
    pcm = torch.empty(B, 128000, dtype=torch.int16, device=dev)
    _lib.call('sad_synth_pcm', 7, 0, B, 128000, _lib.ptr(pcm), _lib.stream_handle(dev))
    out = {}
    for dt in ('bf16', 'bf16x3'):
        eng = Engine(merged_sd('n6'), dev, dtype=dt, micro_batch=256)
        maps = eng.frontend(pcm).clone()
        logits, merged = eng.forward_pcm(pcm)
        out[f'{dt}_maps'] = maps.cpu().numpy()
        out[f'{dt}_stem'] = eng.backbones[0].stem(maps[:64]).float().cpu().numpy()
        out[f'{dt}_merged'] = merged.cpu().numpy()
    small = {}
    for k, v in out.items():
        small[k + '_sha256'] = np.frombuffer(hashlib.sha256(np.ascontiguousarray(v).tobytes()).digest(), np.uint8)
        if not k.endswith('_stem'):
            small[k + '_head'] = v[:2]
    np.savez(sys.argv[1], **small)


if __name__ == '__main__':
    main()
