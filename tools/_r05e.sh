B="python -u bench.py --steps 20 --no-bf16 --no-exact --no-cpu-baseline --no-full-loop --no-input-loop --no-size512"
bash tools/gpu_steps.sh \
 "kern:150:python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_apply_fused.py tests/test_gpu_model.py" \
 "ab_src0:150:SELUNET_FUSE_WGRAD_SRC=0 $B" \
 "ab_src1:150:$B" \
 "ab_src0b:150:SELUNET_FUSE_WGRAD_SRC=0 $B" \
 "ab_src1b:150:$B" \
 "prof:420:BENCH_ARGS='--no-bf16 --no-exact --no-size512 --no-input-loop' bash tools/profile_round.sh r05e"
