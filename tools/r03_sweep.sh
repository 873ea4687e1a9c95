#!/bin/bash
# same-box sweep of the sub-batch / micro-batch settings with the round-3 kernels
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
run() {  # label, env, bench args
  r=$(env $2 timeout -k 10 120 python bench.py --kernels-only --steps 20 $3 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["backbone"]["ms_per_step"])') || exit 1
  echo "$1: $r"
}
for i in 1 2; do
  run default "SAD_X=0" ""
  run fmb64 "SAD_FRONT_MB=64" ""
  run fmb256 "SAD_FRONT_MB=256" ""
  run mb512 "SAD_X=0" "--micro-batch 512"
  run mb2048 "SAD_X=0" "--micro-batch 2048"
done 2>&1 | tee gpurun_out/r03_sweep.log
