#!/bin/bash
# same-box A/B: this session's final tree vs its starting tree (7c2bbb6, abl/libsad_start.so)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/ab_env.sh "start: tree:" 3 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03_session_ab.log
