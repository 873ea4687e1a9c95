#!/bin/bash
# Kernel trace of tools/bench_arch.py for one architecture (GPU box, repo root):
#   bash tools/prof_arch.sh resnet50 [micro-batch]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A=$1; MB=${2:-512}
OUT=gpurun_out/prof_arch_$A
rm -rf $OUT && mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 tools/bench_arch.py --arch $A --micro-batch $MB --steps 2 --warmup 1 > $OUT/trace.log 2>&1 || exit 1
T=$(find $OUT/trace -name 'run_kernel_trace.csv' | head -1 | xargs dirname)
python3 tools/profsum.py --trace $T --steps 3 > $OUT.md
head -30 $OUT.md
