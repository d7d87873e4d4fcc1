B="python -u bench.py --steps 20 --no-bf16 --no-exact --no-cpu-baseline --no-full-loop --no-input-loop --no-size512"
L=$(pwd)/_ab/libselunet_old4ch.so
bash tools/gpu_steps.sh \
 "A:120:SELUNET_LIB=$L SELUNET_FUSE_WGRAD_SRC=64 $B" \
 "B:120:SELUNET_FUSE_WGRAD_SRC=64 $B" \
 "C:120:$B" \
 "A2:120:SELUNET_LIB=$L SELUNET_FUSE_WGRAD_SRC=64 $B" \
 "B2:120:SELUNET_FUSE_WGRAD_SRC=64 $B" \
 "C2:120:$B"
