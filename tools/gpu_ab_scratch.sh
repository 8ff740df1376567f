cd "$GRAFT_REPO_ROOT" || exit 2
export LBM_DEBUG_KNOBS=1
bash tools/gpu_steps.sh \
  "300|res_trace|python3 tools/ab_bench.py --n 1024 --steps 2000 --warmup 100 --rounds 2 --variant bit:LBM_KERNEL=resident,LBM_RES_TRACE=1 --variant tol:FLAGS=4,LBM_KERNEL=resident,LBM_RES_TRACE=1"
grep -h "resident trace\|variant" gpurun_out/res_trace.log | tail -8
