#!/bin/bash
# Same-box A/B of bench.py between abl/libsad_<A>.so and the in-tree libsad.so,
# interleaved (box-to-box DVFS spread is ~10%, so only same-box pairs compare):
#   bash tools/ab_bench.sh base [rounds]
A=$1; N=${2:-2}
for i in $(seq $N); do
  echo "A($A): $(SAD_LIB=abl/libsad_$A.so timeout -k 10 120 python bench.py --kernels-only --steps 20 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["launch_avg_us"], d["roofline"]["backbone"]["ms_per_step"], d["roofline"].get("frontend", {}).get("ms_per_step"))')" || exit 1
  echo "B(tree): $(timeout -k 10 120 python bench.py --kernels-only --steps 20 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["launch_avg_us"], d["roofline"]["backbone"]["ms_per_step"], d["roofline"].get("frontend", {}).get("ms_per_step"))')" || exit 1
done
