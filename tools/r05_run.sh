#!/bin/bash
# One GPU-box pass (repo root): the GPU tests, smoke, the default bench line,
# then the kernel trace + PMC traffic of both modes (tools/profile_bench.sh).
#   bash tools/r05_run.sh TAG [tests|notests]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1
if [ "${2:-tests}" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -3 gpurun_out/${TAG}_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
fi
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
tail -c 600 gpurun_out/${TAG}_bench.json
bash tools/profile_bench.sh ${TAG}_x3 --dtype bf16x3 || exit 1
bash tools/profile_bench.sh ${TAG} || exit 1
head -14 gpurun_out/prof_${TAG}_x3.md
head -14 gpurun_out/prof_${TAG}.md
