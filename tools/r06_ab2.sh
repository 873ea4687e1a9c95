#!/bin/bash
# round 6: bit comparison + GPU tests + same-box A/B (tools/_libsad_base.so vs tools/_libsad_alt.so)
set -o pipefail
bash tools/r06_bits.sh && bash tools/r06_ab.sh
