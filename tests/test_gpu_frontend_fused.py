"""GPU: the experimental one-kernel front end (SAD_FE_FUSED=1 fences / 2
agent-scope stores: fe_mel_db's last workgroup per segment standardises the
segment, csrc/frontend.hip) and the XCD-ordered grid (SAD_FE_XCD_MAP=1) against
the default form, bit for bit.  Since round 6 the default is the frame-major
form (fe_mel_db<IT, true> + fe_normalize_fm, three workgroups per CU, the
transpose in the normalisation); SAD_FE_FM=0 is the staged two-kernel form.  The settings are read once per
process, so child processes compute the alternatives.  Cases: ragged batch
sizes (the XCD-ordered grid is padded to a multiple of 8 segments), the
clamped-dB output, the windows entry point, and a repeated launch (the fused
form's per-segment counters must be left at zero)."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEV = 'cuda:0'
SIZES = (1, 13, 64, 301)
CHILD = r'''
import sys, numpy as np, torch
sys.path[:0] = [{root!r}, {pkg!r}]
from sad import _lib
from sad.engine import FrontEnd
fe = FrontEnd('cuda:0')
out = {{}}
for n in {sizes!r}:
    pcm = torch.empty(n, 128000, dtype=torch.int16, device='cuda:0')
    _lib.call('sad_synth_pcm', 21, 5, n, 128000, _lib.ptr(pcm), _lib.stream_handle(torch.device('cuda:0')))
    for rep in range(2):
        m, db = fe(pcm, want_db=True)
        out[f'map{{n}}_{{rep}}'] = m.cpu().numpy()
        out[f'db{{n}}_{{rep}}'] = db.cpu().numpy()
wf = torch.sin(torch.arange(600000, device='cuda:0', dtype=torch.float32) * 0.01) * 0.3
offs = torch.tensor([0, 1, 4000, 77777, 472000], device='cuda:0', dtype=torch.int64)
out['win'] = fe.windows(wf, offs).cpu().numpy()
np.savez({path!r}, **out)
'''


def _ours():
    from sad import _lib
    from sad.engine import FrontEnd
    fe = FrontEnd(DEV)
    out = {}
    for n in SIZES:
        pcm = torch.empty(n, 128000, dtype=torch.int16, device=DEV)
        _lib.call('sad_synth_pcm', 21, 5, n, 128000, _lib.ptr(pcm), _lib.stream_handle(torch.device(DEV)))
        m, db = fe(pcm, want_db=True)
        out[f'map{n}'] = m.cpu().numpy()
        out[f'db{n}'] = db.cpu().numpy()
    wf = torch.sin(torch.arange(600000, device=DEV, dtype=torch.float32) * 0.01) * 0.3
    offs = torch.tensor([0, 1, 4000, 77777, 472000], device=DEV, dtype=torch.int64)
    out['win'] = fe.windows(wf, offs).cpu().numpy()
    return out


@pytest.mark.parametrize('env', [{'SAD_FE_FUSED': '1'}, {'SAD_FE_FUSED': '2'},
                                 {'SAD_FE_FUSED': '2', 'SAD_FE_XCD_MAP': '1'}, {'SAD_FE_XCD_MAP': '1'},
                                 {'SAD_FE_FM': '0'}])
def test_frontend_forms_equal_default(tmp_path, env):
    for k in ('SAD_FE_FUSED', 'SAD_FE_XCD_MAP', 'SAD_FE_FM'):
        assert k not in os.environ, 'this test runs the default form in-process'
    path = str(tmp_path / 'alt.npz')
    code = CHILD.format(root=ROOT, pkg=os.path.join(ROOT, 'synthetic-audio-detection_amd'), sizes=SIZES, path=path)
    r = subprocess.run([sys.executable, '-c', code], env=dict(os.environ, **env), capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    alt = np.load(path)
    ref = _ours()
    for n in SIZES:
        for rep in range(2):
            assert np.array_equal(alt[f'map{n}_{rep}'], ref[f'map{n}']), (env, n, rep)
            assert np.array_equal(alt[f'db{n}_{rep}'], ref[f'db{n}']), (env, n, rep)
    assert np.array_equal(alt['win'], ref['win'])
