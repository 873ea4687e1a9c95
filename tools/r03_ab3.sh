set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/ab_env.sh "base: tree:" 3 2>&1 | grep -E "base|tree" | tee gpurun_out/r03_ab3.log
