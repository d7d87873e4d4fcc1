bash tools/gpu_steps.sh \
 "layA:200:python -u bench.py --no-bf16 --no-exact --no-cpu-baseline --no-full-loop --no-input-loop --no-size512 --steps 10 --layer-report" \
 "layB:200:SELUNET_FUSE_WGRAD_APPLY=1 python -u bench.py --no-bf16 --no-exact --no-cpu-baseline --no-full-loop --no-input-loop --no-size512 --steps 10 --layer-report" \
 "bias:300:python -u tools/bias_error.py"
