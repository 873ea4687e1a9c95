#!/bin/bash
# variant 31 patch pieces at tap 0: block-conv tests, then end to end vs abl/libsad_base.so
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_blockconv.py > gpurun_out/r03_v31dma2_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03_v31dma2_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh "base: tree:" 3 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03_v31dma2.log
