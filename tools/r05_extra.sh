#!/bin/bash
# Round-5 refresh of the secondary measurements (GPU box, repo root):
# configs[3]'s 1 M-segment shard on one GPU (device-synthesised bf16 and
# bf16x3, host-fed bf16), the trainer step, and the deeper backbones.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 300 python tools/run_1m.py --dtype bf16 > $O/r05_run_1m.json 2> $O/r05_run_1m.err || exit 1
tail -c 400 $O/r05_run_1m.json; echo
timeout -k 10 300 python tools/run_1m.py --dtype bf16 --host-fed > $O/r05_run_1m_hostfed.json 2> $O/r05_run_1m_hostfed.err || exit 1
tail -c 400 $O/r05_run_1m_hostfed.json; echo
timeout -k 10 400 python tools/run_1m.py --dtype bf16x3 > $O/r05_run_1m_bf16x3.json 2> $O/r05_run_1m_bf16x3.err || exit 1
tail -c 400 $O/r05_run_1m_bf16x3.json; echo
timeout -k 10 300 python bench_train.py > $O/r05_bench_train.json 2> $O/r05_bench_train.err || exit 1
tail -c 400 $O/r05_bench_train.json; echo
timeout -k 10 400 python tools/bench_arch.py --arch resnet34 resnet50 resnet101 > $O/r05_bench_arch.jsonl 2> $O/r05_bench_arch.err || exit 1
cat $O/r05_bench_arch.jsonl | cut -c1-300
