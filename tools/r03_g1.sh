set -o pipefail
mkdir -p gpurun_out
cd /root/repo
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_blockconv.py tests/test_gpu_x3.py -k "30 or x3_vs_float64" > gpurun_out/r03_v30_tests.log 2>&1
rc=$?
tail -30 gpurun_out/r03_v30_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u tools/convbench.py --blocks --variants 13 30 --mb 256 1024 --iters 10 --shapes l3.c2+id l3.c2+ds l4.c2+id l4.c2+ds > gpurun_out/r03_v30_convbench.log 2>&1
rc=$?
cat gpurun_out/r03_v30_convbench.log
exit $rc
