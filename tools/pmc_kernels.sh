#!/bin/bash
# Per-kernel SQ counters of one bench step (GPU box, repo root), two passes:
#   bash tools/pmc_kernels.sh TAG  -> gpurun_out/pmc_TAG.md
set -e
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_$TAG; rm -rf $OUT && mkdir -p $OUT
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
B="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $A -d $OUT/a -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --kernels-only "$@" > $OUT/a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc $B -d $OUT/b -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --kernels-only "$@" > $OUT/b.log 2>&1
python3 - "$OUT" > gpurun_out/pmc_$TAG.md <<'PY'
import csv, collections, glob, sys
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + '/*/**/run_counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0].replace('void ', '')[:60]
        agg[k][r['Counter_Name']].append(float(r['Counter_Value']))
names = ['SQ_WAVE_CYCLES', 'SQ_BUSY_CYCLES', 'SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_ACTIVE_INST_VALU',
         'SQ_ACTIVE_INST_LDS', 'SQ_VALU_MFMA_BUSY_CYCLES', 'SQ_INSTS_VALU', 'SQ_INSTS_MFMA', 'SQ_INSTS_LDS', 'SQ_INSTS_SALU',
         'SQ_INSTS_VMEM', 'SQ_WAIT_INST_LDS', 'SQ_LDS_BANK_CONFLICT', 'SQ_LDS_IDX_ACTIVE']
print('| kernel | ' + ' | '.join(n[3:] for n in names) + ' |')
print('|---' * (len(names) + 1) + '|')
for k, d in sorted(agg.items(), key=lambda kv: -sum(kv[1].get('SQ_WAVE_CYCLES', [0]))):
    print(f'| `{k}` | ' + ' | '.join(f'{sum(d[n]) / len(d[n]):.4g}' if d.get(n) else '' for n in names) + ' |')
PY
cat gpurun_out/pmc_$TAG.md
