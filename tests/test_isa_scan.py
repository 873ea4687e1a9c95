"""CPU: libsad.so contains no packed-FP32 VALU instructions (v_pk_fma_f32,
v_pk_mul_f32, v_pk_add_f32).  Round 6 found them returning wrong values on
MI355X when another wave's MFMAs ran on the same CU: the front end computed
single power bins or whole frames wrongly beside the backbone's stem or beside
a kernel of bare MFMA chains, and never beside kernels without MFMAs
(tools/fe_concurrency.py); built without them, none of those
runs differed.  The Makefile turns the instructions off for the device; this
checks the library that ships."""
import os
import sys

import pytest

from conftest import PKG, ROOT

LIB = os.path.join(PKG, 'sad', 'libsad.so')


@pytest.mark.skipif(not os.path.exists('/opt/rocm/lib/llvm/bin/llvm-objdump'), reason='no llvm-objdump')
def test_libsad_has_no_packed_fp32():
    sys.path.insert(0, os.path.join(ROOT, 'tools'))
    import isa_scan
    assert os.path.exists(LIB), 'build libsad.so first'
    counts, n = isa_scan.scan(LIB, r'v_pk_(fma|mul|add)_f32')
    assert n >= 10, f'only {n} gfx950 code objects found in libsad.so'
    assert not counts, f'packed-FP32 instructions in {dict(counts.most_common(5))}'
    # the scanner does see instructions of that family
    mfma, _ = isa_scan.scan(LIB, r'v_mfma_f32_16x16x32_bf16')
    assert sum(mfma.values()) > 1000
