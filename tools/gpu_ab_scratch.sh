cd "$GRAFT_REPO_ROOT" || exit 2
bash tools/gpu_steps.sh "300|t_probe|python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py -k 'placement_probe'"
