#!/bin/bash
# x2 conv forward/dgrad (or ONLY=wgrad: weight gradient) timing (tools/conv_bench.py --x2) under the
# build and every _ab/libselunet_*.so. Run on the GPU box from the repo root; LAYERS / ONLY select.
R=$(cd "$(dirname "$0")/.." && pwd)
for lib in $R/selectivenet_for_semantic_segmentation_binary_amd/libselunet.so $R/_ab/libselunet_*.so; do
  echo "== $(basename $lib)"
  SELUNET_LIB=$lib timeout -k 5 120 python3 $R/tools/conv_bench.py --dtype fp32 --x2 --iters 10 ${ONLY:+--only $ONLY} \
    --layers ${LAYERS:-enc1_2,enc2_2,dec3_1,dec1_1} || exit $?
done
