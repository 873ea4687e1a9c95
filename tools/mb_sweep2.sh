#!/bin/bash
# Same-box micro-batch sweep (bench.py --kernels-only), interleaved rounds:
#   bash tools/mb_sweep2.sh "bf16:512 bf16:1024 bf16x3:256" [rounds] [steps]
N=${2:-2}; ST=${3:-20}
for i in $(seq $N); do
  for cfg in $1; do
    dt=${cfg%%:*}; mb=${cfg#*:}
    r=$(timeout -k 10 300 python bench.py --kernels-only --dtype $dt --steps $ST --micro-batch $mb 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], r["launch_avg_us"], r["achieved"], r["backbone"]["ms_per_step"])') || exit 1
    echo "$cfg: $r"
  done
done
