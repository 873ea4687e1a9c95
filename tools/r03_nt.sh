#!/bin/bash
# variant 31 epilogue: nontemporal 16-B stores (tree) vs plain (abl/libsad_base.so), same box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/ab_conv.sh base "31" "l3.c2+id l4.c2+id" 512 2 2>&1 | tee gpurun_out/r03_nt.log
bash tools/ab_env.sh "base: tree:" 2 2>&1 | tee -a gpurun_out/r03_nt.log
