#!/bin/bash
# Same-box A/B of the split-bf16 bench under env settings, interleaved:
#   bash tools/ab_x3.sh "SAD_X3_RW=0 SAD_X3_RW=1" [rounds]
N=${2:-2}
for i in $(seq $N); do
  for e in $1; do
    r=$(env $e timeout -k 10 300 python bench.py --kernels-only --dtype bf16x3 --steps 8 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])') || exit 1
    echo "$e: $r"
  done
done
