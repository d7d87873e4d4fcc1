B="python -u bench.py --steps 20 --no-bf16 --no-exact --no-cpu-baseline --no-full-loop --no-input-loop --no-size512"
bash tools/gpu_steps.sh \
 "n1:120:$B" \
 "n2:120:SELUNET_FUSE_WGRAD_APPLY=2 $B" \
 "m256:120:SELUNET_FUSE_WGRAD_MAX_CI=256 $B" \
 "m128:120:SELUNET_FUSE_WGRAD_MAX_CI=128 $B" \
 "n1b:120:$B" \
 "n2b:120:SELUNET_FUSE_WGRAD_APPLY=2 $B" \
 "m256b:120:SELUNET_FUSE_WGRAD_MAX_CI=256 $B" \
 "m128b:120:SELUNET_FUSE_WGRAD_MAX_CI=128 $B" \
 "kern:200:python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_fullsize.py"
