#!/bin/bash
# Build variants of libselunet.so with $SRC (default conv3x3) .hip compiled under extra -D flags (the
# other objects shared) into _ab/ for A/B timing with SELUNET_LIB=_ab/libselunet_<name>.so (tools/ab_run.sh).
#   bash tools/ablate.sh "bpf3:-DSELUNET_BPF=3" "early:-DSELUNET_HEARLY=1" "abl5:-DSELUNET_ABL=5"
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/selectivenet_for_semantic_segmentation_binary_amd
rm -rf "$R/_ab" && mkdir -p "$R/_ab"
SRC=${SRC:-conv3x3}
objs=$(ls "$P"/_build/*.o | grep -v $SRC.o)
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $flags -c "$P/csrc/$SRC.hip" \
    -o "$R/_ab/${SRC}_$name.o" &
done
wait
for spec in "$@"; do
  name=${spec%%:*}
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs "$R/_ab/${SRC}_$name.o" -o "$R/_ab/libselunet_$name.so"
  rm "$R/_ab/${SRC}_$name.o"
done
ls "$R/_ab"
