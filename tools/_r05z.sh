bash tools/gpu_steps.sh \
 "suite:900:python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests" \
 "smoke:200:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "bench:400:python -u bench.py" \
 "bs16:150:python -u bench.py --batch 16 --steps 30 --no-bf16 --no-exact --no-cpu-baseline --no-full-loop --no-input-loop --no-size512" \
 "prof:420:BENCH_ARGS='--no-bf16 --no-exact --no-size512 --no-input-loop' bash tools/profile_round.sh r05z"
