#!/bin/bash
# PMC passes over block-conv shapes (run on the GPU box from the repo root):
#   VARIANTS="9 20" SHAPES="l1.c2+id" bash tools/pmc_conv.sh
# then: python tools/pmcdump.py gpurun_out/pmc_conv
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_conv
VARIANTS=${VARIANTS:-"9 13"}
SHAPES=${SHAPES:-"l1.c2+id l4.c2+id"}
rm -rf $OUT && mkdir -p $OUT
run() {  # $1 = pass name, $2 = counters
  timeout -k 10 200 rocprofv3 --pmc $2 -d $OUT/$1 -o run --output-format csv -- \
    python3 tools/convbench.py --blocks --mb 128 --variants $VARIANTS --iters 3 --shapes $SHAPES > $OUT/$1.log 2>&1
}
run p1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
run p2 "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
run p3 "TA_TA_BUSY TA_BUFFER_READ_LDS_WAVEFRONTS TA_DATA_STALLED_BY_TC_CYCLES TA_ADDR_STALLED_BY_TC_CYCLES TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ"
run p4 "TCC_HIT TCC_MISS TCP_TCR_TCP_STALL_CYCLES TD_TD_BUSY SQ_INSTS_SALU SQ_INSTS_VALU"
echo done
