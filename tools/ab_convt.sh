#!/bin/bash
R=$(cd "$(dirname "$0")/.." && pwd)
for lib in $R/selectivenet_for_semantic_segmentation_binary_amd/libselunet.so $R/_ab/libselunet_*.so; do
  echo "== $(basename $lib)"
  SELUNET_LIB=$lib timeout -k 5 60 python3 $R/tools/convt_bench.py || exit $?
done
