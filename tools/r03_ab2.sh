set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_deep_golden.py tests/test_gpu_multirank.py tests/test_gpu_conv_bn_train.py tests/test_gpu_accuracy_gate.py > gpurun_out/r03_ab2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03_ab2_tests.log
bash tools/ab_env.sh "tree:SAD_L1_FUSED=0 tree:SAD_L1_FUSED=1 tree:SAD_L1_FUSED=1,SAD_FRONT_MB=64 tree:SAD_L1_FUSED=1,SAD_FRONT_MB=128 tree:SAD_L1_FUSED=0,SAD_FRONT_MB=64" 2 2>&1 | tee gpurun_out/r03_ab2.log
