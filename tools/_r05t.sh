B="python -u bench.py --steps 20 --no-bf16 --no-exact --no-cpu-baseline --no-full-loop --no-input-loop --no-size512"
L=$(pwd)/_ab/libselunet_oldpool.so
bash tools/gpu_steps.sh \
 "kern:200:python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k pool" \
 "new:120:$B" \
 "old:120:SELUNET_LIB=$L $B" \
 "new2:120:$B" \
 "old2:120:SELUNET_LIB=$L $B"
