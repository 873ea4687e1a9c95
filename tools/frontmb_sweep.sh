#!/bin/bash
# bench.py over SAD_FRONT_MB (stem/layer1/layer2 sub-chunk) values (GPU box, repo root)
set -e
mkdir -p gpurun_out
for f in "$@"; do
  SAD_FRONT_MB=$f timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bfm_$f.log 2>&1
  python - "$f" <<'PY'
import json, sys
f = sys.argv[1]
d = json.loads(open(f'gpurun_out/bfm_{f}.log').read().strip().splitlines()[-1])
print(f"front_mb={f:>4} {d['value']:9.1f} seg/s  {d['ms_per_step']:7.2f} ms/step  backbone frac {d['roofline']['frac']:.3f}")
PY
done
