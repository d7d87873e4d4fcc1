B="python -u bench.py --steps 20 --no-bf16 --no-exact --no-cpu-baseline --no-full-loop --no-input-loop --no-size512"
B16="python -u bench.py --batch 16 --steps 40 --no-bf16 --no-exact --no-cpu-baseline --no-full-loop --no-input-loop --no-size512"
L=$(pwd)/_ab/libselunet_oldgrid.so
bash tools/gpu_steps.sh \
 "kern:200:python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_apply_fused.py tests/test_gpu_kernels.py -k 'pool'" \
 "new16:120:$B16" \
 "old16:120:SELUNET_LIB=$L $B16" \
 "new16b:120:$B16" \
 "old16b:120:SELUNET_LIB=$L $B16" \
 "new:120:$B" \
 "old:120:SELUNET_LIB=$L $B"
