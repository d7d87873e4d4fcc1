#!/bin/bash
# fp32/bf16 conv forward timing (tools/conv_bench.py --only fwd) under every _ab/libselunet_*.so
# variant (tools/ab_build.py). Run on the GPU box from the repo root. DTYPE, LAYERS, ONLY select.
R=$(cd "$(dirname "$0")/.." && pwd)
for lib in $R/_ab/libselunet_*.so; do
  echo "== $(basename $lib)"
  SELUNET_LIB=$lib timeout -k 5 120 python3 $R/tools/conv_bench.py --dtype ${DTYPE:-fp32} --only ${ONLY:-fwd} \
    --iters 5 --layers ${LAYERS:-enc1_2,dec1_2,enc2_2,dec3_1} ${EXTRA:-} || exit $?
done
