cd "$GRAFT_REPO_ROOT" || exit 2
export LBM_DEBUG_KNOBS=1
bash tools/gpu_steps.sh \
  "600|t_3d|python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_d3q19.py -k block_rows" \
  "400|b3d|for v in 12:1 16:0 12:0 12:1 16:0 12:0; do LBM3D_TH=\${v%:*} LBM3D_PD=\${v#*:} python3 tools/bench3d.py --n 512 --steps 20 --rounds 3 || exit 1; done"
grep -h "passed\|failed" gpurun_out/t_3d.log | tail -2; cat gpurun_out/b3d.log | grep grid
