set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03s3_gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r03s3_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03s3_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r03s3_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r03s3_bench.log 2>&1 || exit 1
tail -1 gpurun_out/r03s3_bench.log
