cd "$GRAFT_REPO_ROOT" || exit 2
K="LBM_DEBUG_KNOBS=1"
V=""
for s in 2 3 4 5 6 7 8; do V="$V --variant t$s:FLAGS=4,$K,LBM_TOL_S=$s"; done
for s in 2 3 4 5 6; do V="$V --variant b$s:$K,LBM_STREAM_S=$s"; done
bash tools/gpu_steps.sh "500|ab_spl_ow16|python3 tools/ab_bench.py --n 8192 --steps 840 --warmup 24 --rounds 2 $V"
grep variant gpurun_out/ab_spl_ow16.log | cut -c1-20,110-230
