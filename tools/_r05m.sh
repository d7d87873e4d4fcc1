B="python -u bench.py --steps 20 --no-bf16 --no-exact --no-cpu-baseline --no-full-loop --no-input-loop --no-size512"
bash tools/gpu_steps.sh \
 "kern:200:python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_apply_fused.py tests/test_gpu_model.py" \
 "src1:120:$B" \
 "src0:120:SELUNET_FUSE_WGRAD_SRC=0 $B" \
 "src1b:120:$B" \
 "src0b:120:SELUNET_FUSE_WGRAD_SRC=0 $B"
