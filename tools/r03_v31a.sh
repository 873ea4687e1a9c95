set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/r03_l1b.sh || exit 1
timeout -k 10 400 python -u tools/convbench.py --blocks --variants 31 --mb 1024 --iters 10 --ablate 0 1 2 4 8 --shapes l3.c2+id l4.c2+id > gpurun_out/r03_v31a.log 2>&1 || exit 1
cat gpurun_out/r03_v31a.log
