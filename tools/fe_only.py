"""The front end alone on 2,048 synthetic segments (for a kernel trace): python tools/fe_only.py [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'synthetic-audio-detection_amd')]

import torch  # noqa: E402

from sad import _lib  # noqa: E402
from sad.engine import FrontEnd  # noqa: E402

dev = torch.device('cuda:0')
pcm = torch.empty(2048, 128000, dtype=torch.int16, device=dev)
_lib.call('sad_synth_pcm', 3, 0, 2048, 128000, _lib.ptr(pcm), _lib.stream_handle(dev))
fe = FrontEnd(dev)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 10):
    fe(pcm)
torch.cuda.synchronize()
