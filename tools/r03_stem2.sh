set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for L in base tree; do
  LIB=synthetic-audio-detection_amd/sad/libsad.so; [ $L = base ] && LIB=abl/libsad_base.so
  rm -rf gpurun_out/st_$L
  SAD_LIB=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/st_$L -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --kernels-only > gpurun_out/st_$L.log 2>&1 || exit 1
  f=$(find gpurun_out/st_$L -name 'run_kernel_stats.csv' | head -1)
  echo "== $L"; grep -E "stem|l1block|halo256r|fe_mel" $f | cut -d, -f1-5
done
