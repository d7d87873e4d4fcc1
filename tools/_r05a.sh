bash tools/gpu_steps.sh \
 "kern:300:python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_apply_fused.py tests/test_gpu_overlap.py tests/test_gpu_x2.py tests/test_gpu_kernels.py" \
 "model:300:SELUNET_FUSE_WGRAD_APPLY=1 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_model.py" \
 "benchA:150:python -u bench.py --no-bf16 --no-exact --no-cpu-baseline --no-full-loop --no-input-loop --no-size512 --steps 10" \
 "benchB:150:SELUNET_FUSE_WGRAD_APPLY=1 python -u bench.py --no-bf16 --no-exact --no-cpu-baseline --no-full-loop --no-input-loop --no-size512 --steps 10" \
 "benchTQ:150:SELUNET_FUSE_WGRAD_APPLY=1 SELUNET_TILE_QUEUE=1 python -u bench.py --no-bf16 --no-exact --no-cpu-baseline --no-full-loop --no-input-loop --no-size512 --steps 10" \
 "ovltq:200:python -u tools/overlap_emulation.py --batch 16 --steps 20 --reps 2 --cases 0:0,16:300 --option TILE_QUEUE=1 --json gpurun_out/ovl16_tq.json && python -u tools/overlap_emulation.py --batch 16 --steps 20 --reps 2 --cases 0:0,16:300 --json gpurun_out/ovl16_tq0.json"
cp gpurun_out/summary.txt gpurun_out/summary_a.txt
bash tools/gpu_steps.sh "bias:240:python -u tools/bias_error.py" "biastq:240:SELUNET_TILE_QUEUE=1 python -u tools/bias_error.py"
