#!/bin/bash
# layer2.0's stride-2 conv1 (the only Cout = 128 implicit-GEMM conv left): variant 15 vs 10 vs 19, same box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/ab_env.sh "tree:SAD_C128_VARIANT=15 tree:SAD_C128_VARIANT=10 tree:SAD_C128_VARIANT=19 tree:SAD_C128_VARIANT=12" 2 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03_c128.log
