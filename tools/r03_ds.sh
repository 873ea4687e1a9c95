#!/bin/bash
# variant 41's downsample form: its block-conv cases, then the same-box A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_blockconv.py -k "41 or l2" > gpurun_out/r03_ds_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r03_ds_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh "tree:SAD_L2_DS_RW=0 tree:SAD_L2_DS_RW=1" 3 2>&1 | tee gpurun_out/r03_ds_ab.log
