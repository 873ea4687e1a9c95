set -o pipefail
cd /root/repo; mkdir -p gpurun_out
timeout -k 10 240 python -u tools/convbench.py --blocks --variants 13 30 --mb 256 1024 --iters 10 --shapes l3.c2+id l3.c2+ds l4.c2+id l4.c2+ds > gpurun_out/r03_m1_convbench.log 2>&1 || exit $?
timeout -k 10 240 python -u tools/convbench.py --blocks --variants 13 30 --mb 1024 --iters 10 --shapes l4.c2+id l3.c2+id --ablate 1 2 4 8 16 32 > gpurun_out/r03_m1_ablate.log 2>&1 || exit $?
SAD_LIB=abl/libsad_stamps.so timeout -k 10 120 python -u tools/stamp_v30.py > gpurun_out/r03_m1_stamps.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --no-cpu-baseline --parity-steps 20 > gpurun_out/r03_m1_bench.log 2>&1 || exit $?
cat gpurun_out/r03_m1_convbench.log gpurun_out/r03_m1_ablate.log; grep -v amdgpu.ids gpurun_out/r03_m1_stamps.log | grep -E "^---|stamps|clock M" ; tail -2 gpurun_out/r03_m1_bench.log | cut -c1-1500
