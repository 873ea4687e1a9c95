#!/bin/bash
# Kernel trace + HBM PMC passes of bench.py (GPU box, repo root):
#   bash tools/profile_bench.sh TAG [extra bench args]
# -> gpurun_out/prof_TAG/{trace,fetch,write}, summary gpurun_out/prof_TAG.md
# (per-step figures over 10 backbone passes: 1 warm-up + 3 timed + the timed
# output check's sequential forward + 5 isolated() passes of the overlapped run;
# the side-stream front end adds one front end)
set -e
TAG=$1; shift
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
OUT=gpurun_out/prof_$TAG
rm -rf $OUT && mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 bench.py --steps 3 --warmup 1 --kernels-only "$@" > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- \
  python3 bench.py --steps 1 --warmup 1 --kernels-only "$@" > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- \
  python3 bench.py --steps 1 --warmup 1 --kernels-only "$@" > $OUT/write.log 2>&1
T=$(find $OUT/trace -name 'run_kernel_trace.csv' | head -1 | xargs dirname)
F=$(find $OUT/fetch -name 'run_counter_collection.csv' | head -1 | xargs dirname)
W=$(find $OUT/write -name 'run_counter_collection.csv' | head -1 | xargs dirname)
python3 tools/profsum.py --trace $T --fetch $F --write $W --steps ${PROF_STEPS:-10} --json $OUT.traffic.json > $OUT.md
tail -1 $OUT/trace.log >> $OUT.md
cp $(find $OUT/trace -name 'run_kernel_stats.csv' | head -1) $OUT.stats.csv
