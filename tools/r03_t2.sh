set -o pipefail
cd /root/repo; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_blockconv.py tests/test_gpu_parity.py tests/test_gpu_parity16.py tests/test_gpu_accuracy_gate.py tests/test_gpu_deep_golden.py tests/test_gpu_deep_resnet.py tests/test_gpu_large_batch.py tests/test_gpu_dropin.py -s > gpurun_out/r03_t2.log 2>&1
rc=$?
grep -E "max\||passed|failed|Error|bf16 mb|FAIL" gpurun_out/r03_t2.log | tail -25
[ $rc -eq 0 ] || exit $rc
bash tools/profile_bench.sh r03 > /dev/null 2>&1 || exit 1
head -14 gpurun_out/prof_r03.md
