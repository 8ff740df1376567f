cd "$GRAFT_REPO_ROOT" || exit 2
V=""
for i in 1 2 3 4; do V="$V --variant probe$i:LBM_PLACEMENT_LOG=1 --variant off$i:LBM_PLACEMENT_TRIES=1"; done
bash tools/gpu_steps.sh \
  "400|probe8b|python3 tools/ab_bench.py --n 8192 --steps 1000 --warmup 100 --rounds 1 $V" \
  "300|bench1|LBM_PLACEMENT_LOG=1 python bench.py" \
  "300|bench2|LBM_PLACEMENT_LOG=1 python bench.py --steps 20 --warmup 5" || exit 1
