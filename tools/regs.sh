#!/bin/bash
# Per-kernel register / spill / LDS report of one csrc file (gfx950): bash tools/regs.sh conv3x3.hip
cd "$(dirname "$0")/../selectivenet_for_semantic_segmentation_binary_amd/csrc" || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include -c "$1" -o /tmp/_regs.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk '{sub(/ \[-Rpass[^]]*\]/,"")} /Function Name:/{n=$NF} /VGPRs:/{v=$NF} /AGPRs:/{a=$NF} /ScratchSize/{s=$NF} /LDS Size/{l=$NF; print n, "vgpr", v, "agpr", a, "scratch", s, "lds", l}'
