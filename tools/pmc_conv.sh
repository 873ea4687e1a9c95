#!/bin/bash
# PMC passes over two block-conv shapes (run on the GPU box from the repo root).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_conv
mkdir -p $OUT
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
run() {  # $1 = pass name, $2 = counters
  timeout -k 10 200 rocprofv3 --pmc $2 -d $OUT/$1 -o run --output-format csv -- \
    python3 tools/convbench.py --blocks --mb 128 --variants 9 13 --iters 3 --shapes l1.c2+id l4.c2+id > $OUT/$1.log 2>&1
}
run p1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
run p2 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
run p3 "SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
echo done
