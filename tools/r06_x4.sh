#!/bin/bash
# round 6: four-product split-bf16 in the deep Bottleneck plans -- tests + resnet50 bf16x3 throughput A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_x3.py tests/test_gpu_deep_golden.py tests/test_gpu_deep_resnet.py -s > gpurun_out/x4_tests.log 2>&1 || exit $?
for x4 in 1 0; do
  SAD_DEEP_X4=$x4 timeout -k 10 300 python tools/bench_arch.py --arch resnet50 --dtype bf16x3 --micro-batch 64 \
    >> gpurun_out/x4_arch.jsonl 2> gpurun_out/x4_arch_$x4.err || exit $?
done
