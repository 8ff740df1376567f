# Mid-size grids (2048^2, 4096^2): steps per launch and kernel choice.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
V="--variant t10:FLAGS=4 --variant t8:FLAGS=4,LBM_TOL_S=8 --variant t6:FLAGS=4,LBM_TOL_S=6 --variant t4:FLAGS=4,LBM_TOL_S=4 --variant t3:FLAGS=4,LBM_TOL_S=3 --variant t2:FLAGS=4,LBM_TOL_S=2"
V="$V --variant b6: --variant b4:LBM_STREAM_S=4 --variant b3:LBM_STREAM_S=3 --variant b2:LBM_STREAM_S=2 --variant s2:LBM_KERNEL=step2 --variant v4:LBM_KERNEL=vec4"
STEPS=()
for n in 2048 3072 4096 6144; do
  STEPS+=("300|mid_$n|python3 tools/ab_bench.py --n $n --steps 60 --warmup 6 --rounds 2 $V")
done
bash tools/gpu_steps.sh "${STEPS[@]}" || exit $?
