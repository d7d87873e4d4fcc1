#!/bin/bash
# ConvTranspose2d GEMM timing (tools/convt_bench.py, EXTRA=--x2 for fp32 split-fp16) under the build and
# every _ab/libselunet_*.so; then the build under each SELUNET_GATHER_WGS in $WGS. Run on the GPU box.
R=$(cd "$(dirname "$0")/.." && pwd)
for lib in $R/selectivenet_for_semantic_segmentation_binary_amd/libselunet.so $R/_ab/libselunet_*.so; do
  echo "== $(basename $lib)"
  SELUNET_LIB=$lib timeout -k 5 60 python3 $R/tools/convt_bench.py ${EXTRA:-} || exit $?
done
for w in ${WGS:-}; do
  echo "== SELUNET_GATHER_WGS=$w"
  SELUNET_GATHER_WGS=$w timeout -k 5 60 python3 $R/tools/convt_bench.py ${EXTRA:-} || exit $?
done
