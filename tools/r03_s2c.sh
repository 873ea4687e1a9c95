#!/bin/bash
# variant 32 with hand-counted weight waits: block-conv cases, per-launch times
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_blockconv.py -k "32" > gpurun_out/r03_s2c_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03_s2c_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/convbench.py --blocks --mb 512 --variants 13 15 32 --shapes l2.c1 l3.c1 l4.c1 --iters 10 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03_s2c.log
