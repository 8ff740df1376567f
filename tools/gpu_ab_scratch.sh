cd "$GRAFT_REPO_ROOT" || exit 2
bash tools/gpu_steps.sh \
  "300|t_new|python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_d3q19.py -k 'placement'" \
  "900|t_all|python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests" \
  "300|bench|python bench.py" || exit 1
