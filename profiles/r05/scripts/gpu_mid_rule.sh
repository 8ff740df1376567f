# Size-scaled default segment tiers (lbm_engine.hip guide_for) against the
# fixed round-4 tiers, uniform heights and 48-row tiers, across grid sizes.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
V="--variant t: --variant t_old:LBM_STREAM_GUIDE=144:0.85,48:0.1,16 --variant t_uni:LBM_STREAM_GUIDE=0 --variant t_g48:LBM_STREAM_GUIDE=48:0.85,24:0.1,12"
V="$V --variant b: --variant b_old:LBM_STREAM_GUIDE=96:0.85,32:0.1,10 --variant b_uni:LBM_STREAM_GUIDE=0 --variant b_g48:LBM_STREAM_GUIDE=48:0.85,16:0.1,8"
V=$(echo "$V" | sed 's/--variant t\([a-z_0-9]*\):/--variant t\1:FLAGS=4,/g; s/FLAGS=4,--/FLAGS=4 --/g')
STEPS=()
for g in "2048 2048" "3072 3072" "4096 4096" "4096 8192" "6144 6144" "8192 8192"; do
  set -- $g
  STEPS+=("300|mr_$1x$2|python3 tools/ab_bench.py --n $1 --ny $2 --steps 60 --warmup 6 --rounds 2 $V")
done
bash tools/gpu_steps.sh "${STEPS[@]}" || exit $?
