cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
A="python3 tools/ab_bench.py --n 8192 --steps 98 --warmup 14 --rounds 3 --variant tol:FLAGS=4 --variant bit:"
N="LBM_HIP_LIB=build_var/ntl/liblbm_hip.so"
bash tools/gpu_steps.sh \
  "200|ab_base1|$A" "200|ab_ntl1|$N $A" "200|ab_base2|$A" "200|ab_ntl2|$N $A" || exit $?
grep -H variant gpurun_out/ab_base1.log gpurun_out/ab_ntl1.log gpurun_out/ab_base2.log gpurun_out/ab_ntl2.log
