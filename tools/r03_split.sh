#!/bin/bash
# equal image ranges for launches past 2 GiB: tests touching the split, then end to end vs abl/libsad_base.so
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_blockconv.py tests/test_gpu_multirank.py tests/test_gpu_accuracy_gate.py > gpurun_out/r03_split_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03_split_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh "base: tree:" 3 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03_split.log
