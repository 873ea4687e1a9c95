#!/bin/bash
# per-kernel VGPR/AGPR/scratch/occupancy of one HIP source: bash tools/regs.sh block.hip [filter]
cd "$(dirname "$0")/../synthetic-audio-detection_amd/csrc"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Rpass-analysis=kernel-resource-usage -c "$1" -o /tmp/_regs.o 2>&1 |
  grep -E "Function Name|VGPRs:|AGPRs:|ScratchSize|Occupancy" | sed -E 's/.*remark: *//; s/ \[-Rpass.*//' |
  paste - - - - - | grep -E "${2:-.}" | sed -E 's/Function Name: //; s/VGPRs: /v=/; s/AGPRs: /a=/; s/ScratchSize \[bytes\/lane\]: /scr=/; s/Occupancy \[waves\/SIMD\]: /occ=/' |
  while read n rest; do echo "$(echo $n | c++filt | cut -c1-90) $rest"; done
