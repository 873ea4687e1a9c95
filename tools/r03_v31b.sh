set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_blockconv.py tests/test_gpu_parity.py tests/test_gpu_parity16.py tests/test_gpu_accuracy_gate.py tests/test_gpu_multirank.py > gpurun_out/r03_v31b_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03_v31b_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/convbench.py --blocks --variants 31 --mb 1024 --iters 10 --ablate 0 2 8 --shapes l3.c2+id l4.c2+id > gpurun_out/r03_v31b.log 2>&1 || exit 1
cat gpurun_out/r03_v31b.log
