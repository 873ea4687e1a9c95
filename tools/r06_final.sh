#!/bin/bash
# round 6 final measurement set (GPU box, repo root): kernel trace + HBM PMC
# passes (bf16 and split-bf16), SQ counters, the default bench line, the
# trainer (C1 and --head-loss) and the deeper backbones
set -o pipefail
mkdir -p gpurun_out
bash tools/profile_bench.sh r06f || exit $?
bash tools/profile_bench.sh r06fx3 --dtype bf16x3 --steps 3 || exit $?
bash tools/pmc_kernels.sh r06f > /dev/null || exit $?
timeout -k 10 600 python bench.py > gpurun_out/r06f_bench.json 2> gpurun_out/r06f_bench.err || exit $?
timeout -k 10 300 python bench_train.py > gpurun_out/r06f_bench_train.json 2> gpurun_out/r06f_bench_train.err || exit $?
timeout -k 10 300 python bench_train.py --head-loss > gpurun_out/r06f_bench_train_head_loss.json 2> gpurun_out/r06f_bt2.err || exit $?
timeout -k 10 400 python tools/bench_arch.py --arch resnet34 resnet50 resnet101 resnet152 --micro-batch 512 > gpurun_out/r06f_bench_arch.jsonl 2> gpurun_out/r06f_arch.err || exit $?
timeout -k 10 200 python tools/bench_arch.py --arch resnet50 --dtype bf16x3 --micro-batch 64 >> gpurun_out/r06f_bench_arch.jsonl 2>> gpurun_out/r06f_arch.err
