#!/bin/bash
# variant 41 fragment read-ahead 6 (plain / residual) vs 4: tests, isolated conv, end to end vs abl/libsad_base.so
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_blockconv.py -k 41 > gpurun_out/r03_dq_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03_dq_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_conv.sh base "41" "l2.c1b" 1024 2 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03_dq.log
bash tools/ab_env.sh "base: tree:" 3 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r03_dq.log
