#!/bin/bash
# Same-box bench A/B of library builds / settings, interleaved rounds:
#   bash tools/ab_libs.sh "label=LIBPATH:ENV=V,ENV2=V:--bench-arg ..." [rounds]
# (tokens separated by spaces; fields by ':'); headline mode only.
N=${2:-2}
for i in $(seq $N); do
  for cfg in $1; do
    IFS=':' read -r label rest <<< "$cfg"
    lib=${label#*=}; label=${label%%=*}
    IFS=':' read -r envs args <<< "$rest"
    ev=""; for t in ${envs//,/ }; do ev="$ev $t"; done
    r=$(env SAD_LIB=$lib $ev timeout -k 10 150 python bench.py --kernels-only --steps 20 ${args//,/ } 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], r["launch_avg_us"], r["backbone"]["ms_per_step"], r["frontend"]["ms_per_step"], d["timed_output_check"]["bit_identical"])') || { echo "$label: FAILED"; continue; }
    echo "$label: $r"
  done
done
