B="python -u bench.py --steps 20 --no-bf16 --no-exact --no-cpu-baseline --no-full-loop --no-input-loop --no-size512"
L=$(pwd)/_ab
bash tools/gpu_steps.sh \
 "kern:200:python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_x2.py tests/test_gpu_model.py tests/test_gpu_apply_fused.py" \
 "abA:120:SELUNET_LIB=$L/libselunet_A.so $B" \
 "abB:120:SELUNET_LIB=$L/libselunet_B.so $B" \
 "abC:120:SELUNET_LIB=$L/libselunet_C.so $B" \
 "abA2:120:SELUNET_LIB=$L/libselunet_A.so $B" \
 "abB2:120:SELUNET_LIB=$L/libselunet_B.so $B" \
 "abC2:120:SELUNET_LIB=$L/libselunet_C.so $B"
