#!/bin/bash
# Same-box A/B of convbench block shapes: abl/libsad_<A>.so vs the in-tree build
#   bash tools/ab_conv.sh base "10 13" "l2.c1 l3.c1"
A=$1; V=$2; S=$3
for lib in abl/libsad_$A.so synthetic-audio-detection_amd/sad/libsad.so; do
  echo "== $lib"
  SAD_LIB=$lib timeout -k 10 150 python tools/convbench.py --blocks --mb 128 --variants $V --shapes $S --iters 20 2>&1 | grep -v amdgpu.ids || exit 1
done
