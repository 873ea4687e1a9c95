cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_blockconv.py tests/test_gpu_x3.py -k "44" -x -q --timeout 200 --timeout-method thread 2>&1 | tail -3 || exit 1
timeout -k 10 300 python tools/convbench.py --blocks --mb 1024 --variants 32 44 --shapes l3.c1 l4.c1 --ablate 0 2 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python tools/convbench.py --blocks --split --mb 512 --variants 13 15 44 --shapes l2.c1 l3.c1 l4.c1 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 400 python tools/bench_arch.py --arch resnet34 resnet50 resnet101 resnet152 --micro-batch 512 > gpurun_out/r05_bench_arch_mb512.jsonl 2>/dev/null || exit 1
cut -c1-200 gpurun_out/r05_bench_arch_mb512.jsonl
