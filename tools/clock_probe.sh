#!/bin/bash
# Shader clock and power while the bench's timed loop runs (rocm-smi samples).
timeout -k 10 150 python bench.py --kernels-only --steps 800 > gpurun_out/clock_probe_bench.json 2>/dev/null &
pid=$!
for i in $(seq 40); do
  kill -0 $pid 2>/dev/null || break
  echo "t=$SECONDS $(timeout 20 rocm-smi --showclocks --showpower 2>&1 | grep -E "sclk|Graphics Package Power" | tr -s ' ' | tr '\n' ' ')"
  sleep 0.5
done
wait $pid
