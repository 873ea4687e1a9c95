set -o pipefail
cd /root/repo; mkdir -p gpurun_out
timeout -k 10 400 python -u tools/convbench.py --blocks --variants 13 30 --mb 1024 --iters 10 --ablate 0 512 --shapes l3.c2+id l4.c2+id > gpurun_out/r03_m4_convbench.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/convbench.py --blocks --variants 13 30 --mb 1024 --iters 10 --shapes l3.c2+ds l4.c2+ds >> gpurun_out/r03_m4_convbench.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/convbench.py --blocks --variants 13 30 --mb 1024 --iters 10 --ablate 0 512 --shapes l3.c2+id l4.c2+id >> gpurun_out/r03_m4_convbench.log 2>&1 || exit $?
cat gpurun_out/r03_m4_convbench.log
