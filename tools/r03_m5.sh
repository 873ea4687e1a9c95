set -o pipefail
cd /root/repo; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_blockconv.py tests/test_gpu_x3.py -k "30" > gpurun_out/r03_m5_tests.log 2>&1 || { tail -30 gpurun_out/r03_m5_tests.log; exit 1; }
tail -2 gpurun_out/r03_m5_tests.log
timeout -k 10 400 python -u tools/convbench.py --blocks --variants 13 30 --mb 1024 --iters 10 --ablate 0 1 --shapes l3.c2+id l3.c2+ds l4.c2+id l4.c2+ds > gpurun_out/r03_m5_convbench.log 2>&1 || exit $?
cat gpurun_out/r03_m5_convbench.log
bash tools/pmc_conv2.sh r03b > /dev/null 2>&1 || exit 1
cut -d'|' -f2-3,10-11,13 gpurun_out/pmcc_r03b.md
SAD_LIB=abl/libsad_stamps.so timeout -k 10 120 python -u tools/stamp_v30.py > gpurun_out/r03_m5_stamps.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r03_m5_stamps.log | grep -E "^---|stamps" | grep -A2 "v30"
