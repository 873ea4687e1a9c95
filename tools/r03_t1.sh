set -o pipefail
cd /root/repo; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_accuracy_gate.py tests/test_gpu_conv_bn_train.py tests/test_gpu_deep_golden.py tests/test_gpu_ingest.py -s > gpurun_out/r03_t1.log 2>&1
rc=$?
grep -E "max|passed|failed|Error|fused|PASS|FAIL" gpurun_out/r03_t1.log | tail -40
exit $rc
