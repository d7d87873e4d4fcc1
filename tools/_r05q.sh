B="python -u bench.py --steps 20 --no-bf16 --no-exact --no-cpu-baseline --no-full-loop --no-input-loop --no-size512"
L=$(pwd)/_ab
bash tools/gpu_steps.sh \
 "base:120:$B" \
 "x1:120:SELUNET_LIB=$L/libselunet_x1.so $B" \
 "x1p3:120:SELUNET_LIB=$L/libselunet_x1p3.so $B" \
 "base2:120:$B" \
 "x1b:120:SELUNET_LIB=$L/libselunet_x1.so $B" \
 "x1p3b:120:SELUNET_LIB=$L/libselunet_x1p3.so $B"
