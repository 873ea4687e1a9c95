set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_l1block.py > gpurun_out/r03_l1a_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r03_l1a_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/l1bench.py --n 32 256 --ablate 1 8 9 > gpurun_out/r03_l1a_bench.log 2>&1 || exit 1
cat gpurun_out/r03_l1a_bench.log
