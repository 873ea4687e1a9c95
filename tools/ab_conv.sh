#!/bin/bash
# Same-box A/B of convbench block shapes: abl/libsad_<A>.so vs the in-tree build,
# interleaved over rounds:
#   bash tools/ab_conv.sh A "VARIANTS" "SHAPES" [MB] [ROUNDS] [extra convbench args]
A=$1; V=$2; S=$3; MB=${4:-128}; N=${5:-2}; shift 5; X="$@"
for i in $(seq $N); do
  for lib in abl/libsad_$A.so synthetic-audio-detection_amd/sad/libsad.so; do
    echo "== $lib"
    SAD_LIB=$lib timeout -k 10 150 python tools/convbench.py --blocks --mb $MB --variants $V --shapes $S --iters 20 $X 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
