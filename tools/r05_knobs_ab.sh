#!/bin/bash
# Round 5: the sub-batch / micro-batch knobs re-checked on the final kernels
cd "$GRAFT_REPO_ROOT"
BENCH_ARGS="--dtype bf16x3" bash tools/ab_env.sh "tree: tree:SAD_FRONT_MB=128 tree:--micro-batch=1024 tree:SAD_FRONT_MB=32" 2 || exit 1
bash tools/ab_env.sh "tree: tree:SAD_FRONT_MB=512 tree:SAD_FRONT_MB=128" 2 || exit 1
