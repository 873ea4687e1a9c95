#!/bin/bash
# Same-box A/B of front-end settings: bench.py --kernels-only, interleaved
# rounds; prints value and roofline.frontend ms per setting.
#   bash tools/fe_ab.sh "ENV=.. ENV=..:label" ...
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for spec in "$@"; do
    envs=${spec%%:*}; label=${spec##*:}
    env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 2 --kernels-only > gpurun_out/fe_ab.json 2>/dev/null || exit 1
    python -c "
import json; d=json.loads(open('gpurun_out/fe_ab.json').read().strip().splitlines()[-1])
print('round $r $label', d['value'], 'fe_ms', d['roofline']['frontend']['ms_per_step'], 'bb_ms', d['roofline']['backbone']['ms_per_step'])"
  done
done
