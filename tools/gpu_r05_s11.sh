# round 5: tolerance S = 11 (room made by the in-place shifts: 234 VGPRs, LDS
# 19.7 KB per wave) against S = 10, one process, interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp LBM_DEBUG_KNOBS=1
V="--variant t10:FLAGS=4 --variant t11:FLAGS=4,LBM_TOL_S=11 --variant t9:FLAGS=4,LBM_TOL_S=9"
bash tools/gpu_steps.sh \
  "300|s11_par|python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_tolerance.py -k 'launch or lp or S'" \
  "400|s11_ab110|python3 tools/ab_bench.py --n 8192 --steps 110 --warmup 11 --rounds 4 $V" \
  "300|s11_ab20|python3 tools/ab_bench.py --n 8192 --steps 20 --warmup 5 --rounds 5 $V" || exit $?
grep -h variant gpurun_out/s11_ab110.log gpurun_out/s11_ab20.log
