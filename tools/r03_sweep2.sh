#!/bin/bash
# same-box A/B: front sub-batch 256 and micro-batch 2048 vs the defaults (128 / 1024)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
run() {  # label, env, bench args
  r=$(env $2 timeout -k 10 120 python bench.py --kernels-only --steps 30 $3 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["backbone"]["ms_per_step"])') || exit 1
  echo "$1: $r"
}
for i in 1 2 3; do
  run default "SAD_X=0" ""
  run fmb256 "SAD_FRONT_MB=256" ""
  run fmb256_mb2048 "SAD_FRONT_MB=256" "--micro-batch 2048"
  run fmb512_mb2048 "SAD_FRONT_MB=512" "--micro-batch 2048"
done 2>&1 | tee gpurun_out/r03_sweep2.log
