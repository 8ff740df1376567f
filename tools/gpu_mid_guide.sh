# Mid-size grids: segment tiers (LBM_STREAM_GUIDE) for the stream kernel.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
T="--variant t10:FLAGS=4 --variant t10g64:FLAGS=4,LBM_STREAM_GUIDE=64:0.85,32:0.1,16"
T="$T --variant t10g48:FLAGS=4,LBM_STREAM_GUIDE=48:0.85,24:0.1,12 --variant t8:FLAGS=4,LBM_TOL_S=8"
T="$T --variant t8g64:FLAGS=4,LBM_TOL_S=8,LBM_STREAM_GUIDE=64:0.85,32:0.1,16 --variant t6:FLAGS=4,LBM_TOL_S=6"
T="$T --variant t6g48:FLAGS=4,LBM_TOL_S=6,LBM_STREAM_GUIDE=48:0.85,16:0.1,8"
B="--variant b6: --variant b6g48:LBM_STREAM_GUIDE=48:0.85,16:0.1,8 --variant b6g32:LBM_STREAM_GUIDE=32:0.85,16:0.1,8"
B="$B --variant b6g144:LBM_STREAM_GUIDE=144:0.85,48:0.1,16 --variant s2:LBM_KERNEL=step2"
STEPS=()
for n in 2048 3072 4096; do
  STEPS+=("300|mg_t_$n|python3 tools/ab_bench.py --n $n --steps 60 --warmup 6 --rounds 2 $T")
  STEPS+=("300|mg_b_$n|python3 tools/ab_bench.py --n $n --steps 60 --warmup 6 --rounds 2 $B")
done
bash tools/gpu_steps.sh "${STEPS[@]}" || exit $?
