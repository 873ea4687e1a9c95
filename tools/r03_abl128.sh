#!/bin/bash
# variant 31 with the store-only ablation bit (must be neutral at ablate 0):
# tests, isolated convs and end to end vs abl/libsad_base.so
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_blockconv.py tests/test_gpu_multirank.py tests/test_gpu_parity.py > gpurun_out/r03_abl128_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03_abl128_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_conv.sh base "31" "l3.c2+id l4.c2+ds" 1024 1 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03_abl128.log
bash tools/ab_env.sh "base: tree:" 3 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r03_abl128.log
