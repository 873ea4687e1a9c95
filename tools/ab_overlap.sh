#!/bin/bash
# Same-box A/B of the side-stream front end (bench.py --overlap-frontend 1 / 0),
# headline mode only, interleaved rounds.  Output: gpurun_out/ab_overlap.log
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for ov in 1 0; do
    timeout -k 10 240 python -u bench.py --steps 30 --warmup 3 --kernels-only --overlap-frontend $ov \
      > gpurun_out/ab_ov_${ov}_${r}.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_ov_${ov}_${r}.json')); print('overlap', $ov, 'round', $r, d['value'], d['ms_per_step'], d['timed_output_check']['bit_identical'])" | tee -a gpurun_out/ab_overlap.log
  done
done
