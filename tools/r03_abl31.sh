#!/bin/bash
# variant 31 timing ablations (wrong results): 1 no loads / DMA in the loop,
# 2 no patch DMA, 4 no weight loads, 8 no epilogue
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python tools/convbench.py --blocks --mb 512 --variants 31 --shapes l3.c2+id l4.c2+id --ablate 0 1 2 4 6 8 --iters 10 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03_abl31.log
