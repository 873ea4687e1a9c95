set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_parity16.py tests/test_gpu_accuracy_gate.py tests/test_gpu_deep_golden.py tests/test_gpu_img3.py > gpurun_out/r03_stem_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03_stem_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh "base: tree:" 3 2>&1 | grep -E "base|tree" | tee gpurun_out/r03_stem_ab.log
