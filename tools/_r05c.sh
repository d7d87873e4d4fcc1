bash tools/gpu_steps.sh \
 "suite:900:python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider" \
 "bias:240:python -u tools/bias_error.py"
