cd "$GRAFT_REPO_ROOT" || exit 2
V="--variant w1:FLAGS=4 --variant w2:FLAGS=4,LBM_TOL_CFG=5 --variant w4:FLAGS=4,LBM_TOL_CFG=6 --variant w2s8:FLAGS=4,LBM_TOL_CFG=5,LBM_TOL_S=8 --variant w4s8:FLAGS=4,LBM_TOL_CFG=6,LBM_TOL_S=8"
bash tools/gpu_steps.sh \
  "300|t_mw|python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_tolerance.py -k multiwave" \
  "400|ab_mw|python3 tools/ab_bench.py --n 8192 --steps 98 --warmup 14 --rounds 3 $V" \
  "300|ab_mw20|python3 tools/ab_bench.py --n 8192 --steps 20 --warmup 5 --rounds 3 $V"
grep -h "passed\|failed" gpurun_out/t_mw.log | tail -2; cat gpurun_out/ab_mw.log gpurun_out/ab_mw20.log | grep variant
