bash tools/gpu_steps.sh \
 "kern:120:python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_apply_fused.py tests/test_gpu_model.py" \
 "bench:400:python -u bench.py" \
 "bs16:150:python -u bench.py --batch 16 --steps 30 --no-bf16 --no-exact --no-cpu-baseline --no-full-loop --no-input-loop --no-size512" \
 "prof:420:bash tools/profile_round.sh r05d"
