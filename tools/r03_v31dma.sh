#!/bin/bash
# variant 31: the next chunk's patch pieces spread over taps 1-6 (0) vs all at tap 1 (16) / tap 0 (32)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 300 python tools/convbench.py --blocks --mb 512 --variants 31 --shapes l3.c2+id l4.c2+id l3.c2+ds --ablate 0 16 32 --iters 10 2>&1 | grep -v amdgpu.ids
done | tee gpurun_out/r03_v31dma.log
