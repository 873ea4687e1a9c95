#!/bin/bash
# Same-box A/B of bench_train.py, interleaved (lib: tree or abl/libsad_<tag>.so):
#   bash tools/ab_train.sh "base: tree:" [rounds]
N=${2:-2}
for i in $(seq $N); do
  for cfg in $1; do
    lib=${cfg%%:*}; envs=${cfg#*:}; [ "$envs" = "$cfg" ] && envs=""
    L=synthetic-audio-detection_amd/sad/libsad.so; [ "$lib" != tree ] && L=abl/libsad_$lib.so
    r=$(env SAD_LIB=$L ${envs//,/ } timeout -k 10 300 python bench_train.py --steps 30 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["segments_per_s"], d["roofline"]["frac"])') || exit 1
    echo "$cfg: $r"
  done
done
