bash tools/gpu_steps.sh \
 "suite:900:python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests" \
 "smoke:200:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'"
