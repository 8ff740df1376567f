# Stream-kernel throughput across grid sizes (single domain, AUTO kernel
# choice, tolerance S = 10 and bitwise), 100 steps after 10 warm-up steps.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
STEPS=()
for n in 1024 2048 4096 8192 12288 16384; do
  STEPS+=("240|sweep_$n|python3 tools/ab_bench.py --n $n --steps 100 --warmup 10 --rounds 2 --variant tol:FLAGS=4 --variant bit:")
done
bash tools/gpu_steps.sh "${STEPS[@]}" || exit $?
grep -h variant gpurun_out/sweep_*.log
