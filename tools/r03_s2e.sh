#!/bin/bash
# variant 32 (hand-counted weight waits) end to end: SAD_S2_PATCH=0/1, same box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/ab_env.sh "tree:SAD_S2_PATCH=0 tree:SAD_S2_PATCH=1" 3 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03_s2e.log
