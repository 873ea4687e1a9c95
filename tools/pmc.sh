#!/bin/bash
# One rocprofv3 PMC pass over a kernels-only bench run (GPU box, repo root):
#   bash tools/pmc.sh TAG "COUNTER ..." [extra bench args]
# -> gpurun_out/pmc_TAG.md: per kernel (full template name, grid), the average
#    of each counter per launch; GRBM_GUI_ACTIVE also as the effective clock
#    (sum over 8 XCDs / 8 / kernel duration, MI355X_MICROARCH.md "DVFS give-back").
set -e
TAG=$1; shift
CTRS=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_$TAG; rm -rf $OUT && mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTRS -d $OUT -o run --output-format csv -- \
  python3 bench.py --steps 1 --warmup 1 --kernels-only "$@" > $OUT/run.log 2>&1
python3 tools/pmcsum.py $OUT > gpurun_out/pmc_$TAG.md
cat gpurun_out/pmc_$TAG.md
