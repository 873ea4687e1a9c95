# Round-3 measurement: GPU tests, smoke, default bench line, kernel trace +
# FETCH/WRITE passes (tools/profile_bench.sh) -> gpurun_out/r03j_*
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03j_gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r03j_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03j_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r03j_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r03j_bench.log 2>&1 || exit 1
tail -1 gpurun_out/r03j_bench.log
bash tools/profile_bench.sh r03j > /dev/null 2>&1 || exit 1
head -30 gpurun_out/prof_r03j.md
