set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_l1block.py > gpurun_out/r03_l1c_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03_l1c_tests.log; [ $rc -eq 0 ] || exit $rc
SAD_L1_DMA=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_l1block.py > gpurun_out/r03_l1c_tests_dma.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/l1bench.py --n 32 128 256 --ablate 1 > gpurun_out/r03_l1c_bench.log 2>&1 || exit 1
cat gpurun_out/r03_l1c_bench.log
SAD_L1_DMA=1 timeout -k 10 300 python -u tools/l1bench.py --n 32 128 256 > gpurun_out/r03_l1c_bench_dma.log 2>&1 || exit 1
cat gpurun_out/r03_l1c_bench_dma.log
SAD_LIB=abl/libsad_l1stamps.so timeout -k 10 300 python -u tools/l1bench.py --n 256 > gpurun_out/r03_l1c_stamps.log 2>&1 || exit 1
grep "stamps" gpurun_out/r03_l1c_stamps.log | tail -2
