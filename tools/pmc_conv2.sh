#!/bin/bash
# SQ instruction / cycle counters of the layer4 conv2 (+id) launches of
# variants 13 and 30, with and without DMA (ablate 0 / 1), per kernel:
#   bash tools/pmc_conv2.sh TAG -> gpurun_out/pmcc_TAG.md
set -e
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmcc_$TAG; rm -rf $OUT && mkdir -p $OUT
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
B="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
for ab in 0 1; do
  for p in A B; do
    timeout -s KILL 120 rocprofv3 --pmc ${!p} -d $OUT/$ab$p -o run --output-format csv -- python3 tools/convbench.py --blocks --variants 13 30 --mb 256 --iters 2 --ablate $ab --shapes l4.c2+id > $OUT/$ab$p.log 2>&1
  done
done
python3 - "$OUT" > gpurun_out/pmcc_$TAG.md <<'PY'
import csv, collections, glob, sys
out = sys.argv[1]
names = ['SQ_WAVE_CYCLES', 'SQ_BUSY_CYCLES', 'SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_ACTIVE_INST_VALU',
         'SQ_ACTIVE_INST_LDS', 'SQ_VALU_MFMA_BUSY_CYCLES', 'SQ_INSTS_VALU', 'SQ_INSTS_MFMA', 'SQ_INSTS_LDS', 'SQ_INSTS_SALU',
         'SQ_INSTS_VMEM', 'SQ_WAIT_INST_LDS', 'SQ_LDS_BANK_CONFLICT', 'SQ_LDS_IDX_ACTIVE']
print('| ablate | kernel | ' + ' | '.join(n[3:] for n in names) + ' |')
print('|---' * (len(names) + 2) + '|')
for ab in '01':
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in 'AB':
        for f in glob.glob(f'{out}/{ab}{p}/**/run_counter_collection.csv', recursive=True):
            for r in csv.DictReader(open(f)):
                k = r['Kernel_Name'].split('(')[0].replace('void ', '')[:48]
                if 'conv' not in k and 'halo' not in k:
                    continue
                agg[k][r['Counter_Name']].append(float(r['Counter_Value']))
    for k, d in sorted(agg.items()):
        print(f'| {ab} | `{k}` | ' + ' | '.join(f'{sum(d[n]) / len(d[n]):.4g}' if d.get(n) else '' for n in names) + ' |')
PY
cat gpurun_out/pmcc_$TAG.md
