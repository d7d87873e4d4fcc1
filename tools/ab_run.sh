#!/bin/bash
# Time conv layers (tools/conv_bench.py) under each library in $LIBS (default: the build and every
# _ab/libselunet_*.so). Run on the GPU box from the repo root.
R=$(cd "$(dirname "$0")/.." && pwd)
LAYERS=${LAYERS:-enc2_2,dec3_1,bot4_1}
for lib in $R/selectivenet_for_semantic_segmentation_binary_amd/libselunet.so $R/_ab/libselunet_*.so; do
  echo "== $(basename $lib)"
  SELUNET_LIB=$lib timeout -k 5 60 python3 $R/tools/conv_bench.py --iters 10 --only fwd --layers $LAYERS || exit $?
done
