#!/bin/bash
# bn_bwd_apply timing (tools/apply_bench.py) under the build and every _ab/libselunet_*.so. GPU box, repo root.
R=$(cd "$(dirname "$0")/.." && pwd)
for lib in $R/selectivenet_for_semantic_segmentation_binary_amd/libselunet.so $R/_ab/libselunet_*.so; do
  echo "== $(basename $lib)"
  SELUNET_LIB=$lib timeout -k 5 60 python3 $R/tools/apply_bench.py || exit $?
done
