cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
V="--variant w1:FLAGS=4 --variant w4:FLAGS=4,LBM_TOL_CFG=5 --variant w8:FLAGS=4,LBM_TOL_CFG=6"
bash tools/gpu_steps.sh \
  "300|t_mw|python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_tolerance.py -k multiwave" \
  "400|ab_mw|python3 tools/ab_bench.py --n 8192 --steps 98 --warmup 14 --rounds 3 $V" \
  "300|ab_mw20|python3 tools/ab_bench.py --n 8192 --steps 20 --warmup 5 --rounds 3 $V" || exit $?
for v in "w1:FLAGS=4" "w4:FLAGS=4,LBM_TOL_CFG=5" "w8:FLAGS=4,LBM_TOL_CFG=6"; do
  n="${v%%:*}"; mkdir -p gpurun_out/pmc_mw/$n
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_mw/$n -o run --output-format csv -- \
    python3 tools/ab_bench.py --n 8192 --steps 42 --warmup 7 --rounds 1 --variant "$v" > gpurun_out/pmc_mw/$n/log.txt 2>&1 || { echo "pmc $n failed"; exit 3; }
done
grep -h "passed\|failed" gpurun_out/t_mw.log | tail -2; cat gpurun_out/ab_mw.log gpurun_out/ab_mw20.log | grep variant
