# Grids between the resident kernel's 1 M cells and the stream kernel's
# 4 M-cell AUTO threshold: AUTO's choice against the stream kernel.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
V="--variant b_auto: --variant b_stream:LBM_KERNEL=stream --variant t_auto:FLAGS=4 --variant t_stream:FLAGS=4,LBM_KERNEL=stream"
STEPS=()
for n in 1024 1280 1536 1792 2048; do
  STEPS+=("240|sm_$n|python3 tools/ab_bench.py --n $n --steps 60 --warmup 6 --rounds 2 $V")
done
bash tools/gpu_steps.sh "${STEPS[@]}" || exit $?
