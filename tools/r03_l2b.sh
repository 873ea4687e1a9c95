set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_blockconv.py -k "41" > gpurun_out/r03_l2b_t1.log 2>&1
rc=$?; tail -15 gpurun_out/r03_l2b_t1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_blockconv.py tests/test_gpu_parity.py tests/test_gpu_parity16.py tests/test_gpu_accuracy_gate.py tests/test_gpu_deep_resnet.py tests/test_gpu_conv_bn_train.py > gpurun_out/r03_l2b_t2.log 2>&1
rc=$?; tail -3 gpurun_out/r03_l2b_t2.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh "tree:SAD_L2_RW=0 tree:SAD_L2_RW=1" 3 2>&1 | grep tree: | tee gpurun_out/r03_l2b_ab.log
