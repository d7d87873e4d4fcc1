B="python -u bench.py --steps 20 --no-bf16 --no-exact --no-cpu-baseline --no-full-loop --no-input-loop --no-size512"
bash tools/gpu_steps.sh \
 "r1:120:$B" \
 "r4:120:SELUNET_BN_FLAG_RATIO=4 $B" \
 "r16:120:SELUNET_BN_FLAG_RATIO=16 $B" \
 "r1b:120:$B" \
 "r4b:120:SELUNET_BN_FLAG_RATIO=4 $B" \
 "r16b:120:SELUNET_BN_FLAG_RATIO=16 $B" \
 "kern16:300:SELUNET_BN_FLAG_RATIO=16 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_fullsize.py tests/test_gpu_train.py"
