#!/bin/bash
# Front-end kernels alone (tools/fe_only.py, 2,048 segments x 10) under rocprofv3 for
# tools/_libsad_base.so and tools/_libsad_alt.so, interleaved: average us per kernel.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for r in 1 2; do
  for L in base alt; do
    O=gpurun_out/fecmp_${L}_$r; rm -rf $O
    SAD_LIB=tools/_libsad_$L.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- \
      python3 tools/fe_only.py 10 > $O.log 2>&1 || exit 1
    S=$(find $O -name 'run_kernel_stats.csv' | head -1)
    python3 - "$S" "$L" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'fe_' in r['Name']:
        print(sys.argv[2], r['Name'].split('(')[0][:48], r['Calls'], round(float(r['AverageNs']) / 1000, 1))
PY
  done
done
