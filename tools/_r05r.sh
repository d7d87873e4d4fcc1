B="python -u bench.py --steps 20 --no-bf16 --no-exact --no-cpu-baseline --no-full-loop --no-input-loop --no-size512"
L=$(pwd)/_ab
bash tools/gpu_steps.sh \
 "kern:200:SELUNET_LIB=$L/libselunet_p1early.so python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_apply_fused.py" \
 "base:120:$B" \
 "p1:120:SELUNET_LIB=$L/libselunet_p1early.so $B" \
 "base2:120:$B" \
 "p1b:120:SELUNET_LIB=$L/libselunet_p1early.so $B"
