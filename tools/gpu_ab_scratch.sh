cd "$GRAFT_REPO_ROOT" || exit 2
bash tools/gpu_steps.sh \
  "300|t_probe3d|python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_d3q19.py -k 'probe or slab'" \
  "400|d3spread|LBM_DEBUG_KNOBS=1 LBM_PLACEMENT_LOG=1 python3 tools/d3_spread.py --engines 6"
grep -h "passed\|failed" gpurun_out/t_probe3d.log | tail -2; cat gpurun_out/d3spread.log | grep "engine\|probe"
