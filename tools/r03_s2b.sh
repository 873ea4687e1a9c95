#!/bin/bash
# per-launch times of the stride-2 convs: implicit GEMM (13 / 15) vs variant 32
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python tools/convbench.py --blocks --mb 256 512 --variants 13 15 32 --shapes l2.c1 l3.c1 l4.c1 --iters 10 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03_s2b.log
