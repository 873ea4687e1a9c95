#!/bin/bash
# variant 31 epilogue ablations: 8 no epilogue, 128 conversion + permutes but no stores
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python tools/convbench.py --blocks --mb 1024 --variants 31 --shapes l3.c2+id l4.c2+ds --ablate 0 8 128 --iters 10 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03_epi.log
