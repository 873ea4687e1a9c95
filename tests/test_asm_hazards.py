"""CPU: the inline-asm MFMA kernels' generated gfx950 code has no compiler
instruction reading or overwriting an asm MFMA's result within its 12 wait
states (tools/asm_hazards.py).  hipcc pads only the MFMAs it
generates itself; a register copy its allocator inserts after an asm MFMA reads
a stale accumulator silently -- round 4 found exactly that in the split-bf16
layer1 kernel (variant 42: the last fragment of a chunk lost its W_hi.X_lo
product), which GPU tests then confirmed (4.8e-4 relative error)."""
import os
import sys

import pytest

from conftest import PKG, ROOT


@pytest.mark.parametrize('src', ['l1block.hip', 'l2conv.hip', 'l2s2conv.hip'])
def test_no_mfma_result_hazards(src):
    sys.path.insert(0, os.path.join(ROOT, 'tools'))
    import asm_hazards
    assert asm_hazards.main([os.path.join(PKG, 'csrc', src)]) == 0
