#!/bin/bash
# Time conv layers (tools/conv_bench.py) with and without an environment switch: ab_env.sh VAR
# (runs VAR unset, then VAR=0). Run on the GPU box from the repo root; LAYERS/ONLY select layers.
R=$(cd "$(dirname "$0")/.." && pwd)
LAYERS=${LAYERS:-enc1_2,enc2_1,dec1_1,dec1_2}
for v in 1 0; do
  echo "== $1=$v"
  env $1=$v timeout -k 5 90 python3 $R/tools/conv_bench.py --iters 10 ${ONLY:+--only $ONLY} --layers $LAYERS || exit $?
done
