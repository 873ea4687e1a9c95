#!/bin/bash
# bench.py over (SAD_FRONT_MB, --micro-batch) pairs on one box: bash tools/frontmb_ab.sh "32:128 16:128 32:256"
for pair in $1; do
  f=${pair%%:*}; m=${pair##*:}
  echo "FRONT_MB=$f mb=$m: $(SAD_FRONT_MB=$f timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --micro-batch $m | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["backbone"]["ms_per_step"], d["roofline"]["launch_avg_us"])')" || exit 1
done
