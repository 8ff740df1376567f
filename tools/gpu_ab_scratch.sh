cd "$GRAFT_REPO_ROOT" || exit 2
bash tools/gpu_steps.sh \
  "600|t_new|python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_tolerance.py tests/test_gpu_parity.py -k 'tolerance or remainder or segments or forced_exchange or large_grid'" \
  "400|ab96|python3 tools/ab_bench.py --n 8192 --steps 96 --warmup 12 --rounds 3 --variant base: --variant s5:LBM_STREAM_S=5 --variant tol6:FLAGS=4 --variant tol7:FLAGS=4,LBM_TOL_S=7 --variant tol8:FLAGS=4,LBM_TOL_S=8" \
  "300|ab20|python3 tools/ab_bench.py --n 8192 --steps 20 --warmup 5 --rounds 3 --variant s5:LBM_STREAM_S=5 --variant tol5:FLAGS=4,LBM_TOL_S=5 --variant tol7:FLAGS=4,LBM_TOL_S=7 --variant tol8:FLAGS=4,LBM_TOL_S=8"
grep -h "passed\|failed" gpurun_out/t_new.log | tail -3; cat gpurun_out/ab96.log gpurun_out/ab20.log | grep variant
