#!/bin/bash
# Round-end measurement on the GPU box (repo root): GPU tests, smoke, the
# default bench line and the trainer bench -> gpurun_out/final_*.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/final_gpu_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/final_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py 2>/dev/null | tail -n1 > gpurun_out/final_bench.json || exit 1
timeout -k 10 300 python bench_train.py --steps 30 2>/dev/null | tail -n1 > gpurun_out/final_bench_train.json || exit 1
