#!/bin/bash
# variant 32 (stride-2 patch-resident): its block-conv cases, the model-level
# GPU tests, then the same-box A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_blockconv.py -k "32 or s2" > gpurun_out/r03_s2_tests.log 2>&1
rc=$?; tail -12 gpurun_out/r03_s2_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh "tree:SAD_S2_PATCH=0 tree:SAD_S2_PATCH=1" 2 2>&1 | tee gpurun_out/r03_s2_ab.log
