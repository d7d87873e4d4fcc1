B="python -u bench.py --steps 20 --no-bf16 --no-exact --no-cpu-baseline --no-full-loop --no-input-loop --no-size512"
L=$(pwd)/_ab/libselunet_ks3.so
bash tools/gpu_steps.sh \
 "base:120:$B" \
 "ks3:120:SELUNET_LIB=$L $B" \
 "base2:120:$B" \
 "ks3b:120:SELUNET_LIB=$L $B"
