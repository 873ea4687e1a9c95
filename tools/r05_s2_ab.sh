#!/bin/bash
# Round 5: variant 44 (stride-2 conv1 of layer3/4, four parity planes) against
# variant 32 (bf16) and the split implicit GEMM (bf16x3), end to end, same box.
cd "$GRAFT_REPO_ROOT"
bash tools/ab_env.sh "tree:SAD_S2_PATCH=1 tree:SAD_S2_PATCH=2" 3 || exit 1
BENCH_ARGS="--dtype bf16x3" bash tools/ab_env.sh "tree:SAD_X3_S2=0 tree:SAD_X3_S2=44" 3 || exit 1
