#!/bin/bash
# Kernel trace of bench_train.py (GPU box, repo root) -> per-step breakdown.
# Extra arguments go to bench_train.py (e.g. --head-loss); OUT names the output.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/prof_train}
rm -rf $OUT && mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 bench_train.py --steps 10 --warmup 3 "$@" > $OUT/trace.log 2>&1 || exit 1
T=$(find $OUT/trace -name 'run_kernel_trace.csv' | head -1)
python3 tools/train_prof.py $T > $OUT.md
cat $OUT.md
