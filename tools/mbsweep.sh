#!/bin/bash
# End-to-end bench over micro-batch sizes (GPU box, repo root):  bash tools/mbsweep.sh 32 64 128
set -e
mkdir -p gpurun_out
for mb in "$@"; do
  timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --micro-batch $mb > gpurun_out/bmb_$mb.log 2>&1
  python - "$mb" <<'PY'
import json, sys
mb = sys.argv[1]
d = json.loads(open(f'gpurun_out/bmb_{mb}.log').read().strip().splitlines()[-1])
print(f"mb={mb:>4} {d['value']:9.1f} seg/s  {d['ms_per_step']:7.2f} ms/step  backbone frac {d['roofline']['frac']:.3f}")
PY
done
