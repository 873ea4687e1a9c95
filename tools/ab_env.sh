#!/bin/bash
# Same-box bench runs of labelled (lib, env) configurations, interleaved:
#   bash tools/ab_env.sh "base:SAD_FRONT_MB=0 tree:SAD_FRONT_MB=32" [rounds]
# (BENCH_ARGS="--dtype bf16x3" times the parity mode instead; a token starting
# with -- is a bench argument of that configuration: "tree:--micro-batch=2048");
# prints seg/s, dominant launch us, backbone ms, front-end ms, held sclk MHz
N=${2:-2}
for i in $(seq $N); do
  for cfg in $1; do
    lib=${cfg%%:*}; envs=${cfg#*:}; [ "$envs" = "$cfg" ] && envs=""
    L=synthetic-audio-detection_amd/sad/libsad.so; [ "$lib" != tree ] && L=abl/libsad_$lib.so
    ev=""; args=""
    for t in ${envs//,/ }; do case "$t" in --*) args="$args $t";; *) ev="$ev $t";; esac; done
    r=$(env SAD_LIB=$L $ev timeout -k 10 120 python bench.py --kernels-only --steps 20 $BENCH_ARGS $args | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], r["launch_avg_us"], r["backbone"]["ms_per_step"], r.get("frontend", {}).get("ms_per_step"), (r.get("clock") or {}).get("sclk_mhz_median"))') || exit 1
    echo "$cfg: $r"
  done
done
