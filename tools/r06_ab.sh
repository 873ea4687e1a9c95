#!/bin/bash
# round 6: same-box A/B of library builds (tools/_libsad_base.so vs tools/_libsad_alt.so) + GPU tests on the alt build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  ${AB_TESTS:-tests/test_gpu_parity.py tests/test_gpu_x3.py tests/test_gpu_img3.py tests/test_gpu_stem_train.py tests/test_gpu_train.py tests/test_gpu_accuracy_gate.py} > gpurun_out/ab_tests.log 2>&1 || exit $?
timeout -k 10 900 bash tools/ab_libs.sh "${AB_CFGS:-base=tools/_libsad_base.so alt=tools/_libsad_alt.so}" ${AB_ROUNDS:-3} > gpurun_out/ab.log 2>&1
