set -o pipefail
cd /root/repo; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_blockconv.py -k "30" > gpurun_out/r03_m7_tests.log 2>&1 || { tail -30 gpurun_out/r03_m7_tests.log; exit 1; }
tail -2 gpurun_out/r03_m7_tests.log
timeout -k 10 400 python -u tools/convbench.py --blocks --variants 13 30 31 --mb 1024 --iters 10 --ablate 0 --shapes l3.c2+id l3.c2+ds l4.c2+id l4.c2+ds > gpurun_out/r03_m7_convbench.log 2>&1 || exit $?
cat gpurun_out/r03_m7_convbench.log
timeout -k 10 400 python -u tools/convbench.py --blocks --variants 31 --mb 1024 --iters 10 --ablate 1 8 --shapes l3.c2+id l4.c2+id > gpurun_out/r03_m7_ablate.log 2>&1 || exit $?
cat gpurun_out/r03_m7_ablate.log
bash tools/ab_env.sh "tree:SAD_HALO256=0 tree:SAD_HALO256=1 tree:SAD_HALO256=2" 2 2>&1 | tee gpurun_out/r03_m7_ab.log || exit 1
