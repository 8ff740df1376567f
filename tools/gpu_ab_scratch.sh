cd "$GRAFT_REPO_ROOT" || exit 2
bash tools/gpu_steps.sh "300|t_probe|LBM_PLACEMENT_LOG=1 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py -k 'placement_probe or forced_exchange'"
grep -h "placement probe\|passed\|failed" gpurun_out/t_probe.log | tail -8
