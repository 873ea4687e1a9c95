#!/bin/bash
# round 6: outputs of tools/_libsad_base.so vs the current build, bit for bit (tools/lib_bits.py);
# BITS_ENV: environment for the current build's run (e.g. SAD_FE_FM=1)
set -o pipefail
mkdir -p gpurun_out
SAD_LIB=tools/_libsad_base.so timeout -k 10 300 python tools/lib_bits.py gpurun_out/bits_base.npz && \
env $BITS_ENV timeout -k 10 300 python tools/lib_bits.py gpurun_out/bits_new.npz
