#!/bin/bash
# fp32 weight-gradient timing (tools/conv_bench.py --only wgrad) and its kernel tests under every
# _ab/libselunet_*.so variant (tools/ab_build.py). Run on the GPU box from the repo root.
R=$(cd "$(dirname "$0")/.." && pwd)
LAYERS=${LAYERS:-enc1_2,enc2_2,enc3_2,dec3_2,dec1_2}
for lib in $R/_ab/libselunet_*.so; do
  echo "== $(basename $lib)"
  SELUNET_LIB=$lib timeout -k 5 120 python3 -m pytest -q -x --timeout 60 --timeout-method thread \
    $R/tests/test_gpu_kernels.py -k "test_conv3x3_wgrad or ws_to" 2>&1 | tail -1 || exit $?
  SELUNET_LIB=$lib timeout -k 5 120 python3 $R/tools/conv_bench.py --dtype fp32 --only wgrad --iters 5 \
    --layers $LAYERS || exit $?
done
