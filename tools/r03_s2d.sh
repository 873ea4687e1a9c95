#!/bin/bash
# variant 32 timing ablations (wrong results): 2 no patch DMA, 4 no weight loads, 8 no epilogue
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python tools/convbench.py --blocks --mb 512 --variants 32 --shapes l2.c1 l3.c1 --ablate 0 2 4 6 8 14 --iters 10 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03_s2d.log
