#!/bin/bash
# Time conv layers (tools/conv_bench.py) with an environment switch unset and set:
#   ab_env.sh VAR=VALUE     (LAYERS / ONLY select layers and fwd|dgrad). Run on the GPU box.
R=$(cd "$(dirname "$0")/.." && pwd)
for e in "" "$1"; do
  echo "== ${e:-baseline}"
  env $e timeout -k 5 120 python3 $R/tools/conv_bench.py --iters 10 ${ONLY:+--only $ONLY} ${LAYERS:+--layers $LAYERS} || exit $?
done
