#!/bin/bash
# Same-box A/B of the split-bf16 bench, interleaved (lib: tree or abl/libsad_<tag>.so):
#   bash tools/ab_x3.sh "base: tree: tree:SAD_X3_RW=0" [rounds] [dtype] [steps]
N=${2:-2}; DT=${3:-bf16x3}; ST=${4:-8}
for i in $(seq $N); do
  for cfg in $1; do
    lib=${cfg%%:*}; envs=${cfg#*:}; [ "$envs" = "$cfg" ] && envs=""
    L=synthetic-audio-detection_amd/sad/libsad.so; [ "$lib" != tree ] && L=abl/libsad_$lib.so
    r=$(env SAD_LIB=$L ${envs//,/ } timeout -k 10 300 python bench.py --kernels-only --dtype $DT --steps $ST 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])') || exit 1
    echo "$cfg: $r"
  done
done
