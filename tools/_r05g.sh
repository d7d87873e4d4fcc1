B="python -u bench.py --steps 20 --no-bf16 --no-exact --no-cpu-baseline --no-full-loop --no-input-loop --no-size512"
bash tools/gpu_steps.sh \
 "kern:200:python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_apply_fused.py tests/test_gpu_x2.py" \
 "kern64:200:SELUNET_WGRAD_BN_BI=1 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_apply_fused.py tests/test_gpu_model.py" \
 "bi128:120:$B" \
 "bi64:120:SELUNET_WGRAD_BN_BI=1 $B" \
 "bi128b:120:$B" \
 "bi64b:120:SELUNET_WGRAD_BN_BI=1 $B"
