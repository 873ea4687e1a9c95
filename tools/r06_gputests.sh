#!/bin/bash
# round 6: the whole GPU suite (one process), then the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
