set -o pipefail
cd /root/repo; mkdir -p gpurun_out
SAD_LIB=abl/libsad_stamps.so timeout -k 10 120 python -u tools/stamp_v30.py > gpurun_out/r03_v30_stamps.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/convbench.py --blocks --variants 13 30 --mb 256 --iters 10 --shapes l4.c2+id --ablate 0 1 2 4 8 16 32 > gpurun_out/r03_v30_ablate.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r03_v30_stamps.log; cat gpurun_out/r03_v30_ablate.log
