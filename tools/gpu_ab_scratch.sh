cd "$GRAFT_REPO_ROOT" || exit 2
V="--variant lp:FLAGS=4 --variant lpnt:FLAGS=4,LBM_TOL_CFG=7"
bash tools/gpu_steps.sh \
  "400|ab_nt|python3 tools/ab_bench.py --n 8192 --steps 98 --warmup 14 --rounds 4 --check $V" \
  "300|ab_nt20|python3 tools/ab_bench.py --n 8192 --steps 20 --warmup 5 --rounds 4 $V"
cat gpurun_out/ab_nt.log gpurun_out/ab_nt20.log | grep variant
