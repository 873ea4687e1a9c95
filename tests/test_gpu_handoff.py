"""GPU: cross-stream hand-offs and concurrency.

Round 5 saw the pipelined bench (the next step's front end on a side stream
during this step's backbone) produce wrong logits in some steps and took it for
a cross-queue hand-off hole.  Round 6 located it (tools/handoff_study.py with
HANDOFF_LOCATE=1, tools/fe_concurrency.py): the dispatch and barrier packets
carry the right fence scopes, and the wrong values were in the MAPS, computed
by the front end while MFMAs of another kernel ran on the same CUs.  A kernel
of bare MFMA chains does it too, a kernel of DPP / ds_bpermute / LDS traffic
does not, and a front end built without packed-FP32 instructions
(v_pk_fma/mul/add_f32) never does: libsad is built without them
(csrc/Makefile NOPK; tests/test_isa_scan.py checks the library).

  * test_frontend_under_concurrent_stem: the case that failed, once, at a
    batch where the packed-FP32 build failed almost surely.
  * test_side_stream_handoffs: libsad consumers of tensors written on a torch
    side stream (as NCCL's stream hands back all-gathered logits or
    all-reduced gradients) after an event wait: the heads/merge, AdamW and the
    backbone, each bit for bit against the sequential result.
"""
import pytest
import torch

from conftest import merged_sd

pytestmark = pytest.mark.gpu

DEV = torch.device('cuda:0')


def _synth(n, seed):
    from sad import _lib
    pcm = torch.empty(n, 128000, dtype=torch.int16, device=DEV)
    _lib.call('sad_synth_pcm', seed, 0, n, 128000, _lib.ptr(pcm), _lib.stream_handle(DEV))
    return pcm


@pytest.fixture(scope='module')
def eng():
    from sad.engine import Engine
    return Engine(merged_sd('n6'), DEV, dtype='bf16', micro_batch=256)


def test_frontend_under_concurrent_stem(eng):
    """The front end (in place, as the bench runs it) while the bf16 stem runs
    on a side stream over as many segments, against a quiet run, bit for bit."""
    B = 1024
    pcm = _synth(B, 3)
    fe, bb = eng.frontend, eng.backbones[0]
    ref = fe(pcm).clone()
    bmaps = fe(_synth(B, 4))
    out = torch.empty_like(ref)
    side = torch.cuda.Stream(DEV)
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        bb.stem(bmaps)  # 1,024 segments of stem work, launched first
    fe(pcm, out=out)
    torch.cuda.synchronize()
    d = out != ref
    where = d.nonzero()[:4].tolist()
    assert not d.any(), f'{int(d.sum())} map values differ under a concurrent stem, e.g. (seg, mel, frame) {where}'


def test_side_stream_handoffs(eng):
    """Tensors produced on a side stream, then an event wait on the consumer's
    stream, then the libsad consumer: the same bits as the sequential run."""
    from sad import _lib
    side = torch.cuda.Stream(DEV)
    cur = torch.cuda.current_stream(DEV)
    g = torch.Generator(device=DEV).manual_seed(11)

    def produced(src):
        """src copied into a fresh tensor on the side stream (the collective's
        output buffer), with the event the consumer waits on."""
        dst = torch.empty_like(src)
        side.wait_stream(cur)  # src is ready
        with torch.cuda.stream(side):
            dst.copy_(src)
            ev = torch.cuda.Event()
            ev.record(side)
        dst.record_stream(cur)
        return dst, ev

    # 1) heads + merge on gathered pooled features
    feats = torch.randn(2048, 512, device=DEV, generator=g).abs_()
    ref_logits, ref_merged = [t.clone() for t in eng.heads([feats])]
    f2, ev = produced(feats)
    cur.wait_event(ev)
    logits, merged = eng.heads([f2])
    torch.cuda.synchronize()
    assert torch.equal(logits, ref_logits) and torch.equal(merged, ref_merged)

    # 2) AdamW on all-reduced gradients
    n = 1 << 22
    p0 = torch.randn(n, device=DEV, generator=g)
    grad = torch.randn(n, device=DEV, generator=g) * 1e-2
    outs = []
    for gsrc in ('seq', 'side'):
        p, m, v = p0.clone(), torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
        gg = grad
        if gsrc == 'side':
            gg, ev = produced(grad)
            cur.wait_event(ev)
        for step in (1, 2):
            _lib.call('sad_adamw_run', _lib.ptr(p), _lib.ptr(gg), _lib.ptr(m), _lib.ptr(v), n, 1e-3, 0.9, 0.999,
                      1e-8, 0.01, step, _lib.stream_handle(DEV))
        outs.append((p, m, v))
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(*outs))

    # 3) the backbone on maps produced on the side stream
    maps = eng.frontend(_synth(512, 5))
    bb = eng.backbones[0]
    ref = bb(maps).clone()
    m2, ev = produced(maps)
    cur.wait_event(ev)
    got = bb(m2)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
