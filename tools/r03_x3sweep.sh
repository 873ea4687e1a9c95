#!/bin/bash
# parity mode (bf16x3): front sub-batch sweep, same box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
run() {
  r=$(env $2 timeout -k 10 200 python bench.py --kernels-only --dtype bf16x3 --steps 10 --warmup 2 $3 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["backbone"]["ms_per_step"])') || exit 1
  echo "$1: $r"
}
for i in 1 2; do
  run fmb32 "SAD_FRONT_MB=32" ""
  run fmb64 "SAD_FRONT_MB=64" ""
  run fmb128 "SAD_FRONT_MB=128" ""
done 2>&1 | tee gpurun_out/r03_x3sweep.log
