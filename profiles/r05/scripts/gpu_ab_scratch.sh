cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp LBM_DEBUG_KNOBS=1
V="--variant g144:FLAGS=4 --variant g144_8:FLAGS=4,LBM_STREAM_GUIDE=144:0.85,48:0.1,16:0.03,8 --variant g160:FLAGS=4,LBM_STREAM_GUIDE=160:0.85,48:0.1,16 --variant g144_64:FLAGS=4,LBM_STREAM_GUIDE=144:0.8,64:0.1,24:0.07,8 --variant g176_8:FLAGS=4,LBM_STREAM_GUIDE=176:0.8,56:0.12,16:0.05,8"
bash tools/gpu_steps.sh \
  "400|ab_g98|python3 tools/ab_bench.py --n 8192 --steps 98 --warmup 14 --rounds 3 $V" \
  "300|ab_g20|python3 tools/ab_bench.py --n 8192 --steps 20 --warmup 5 --rounds 5 $V" || exit $?
cat gpurun_out/ab_g98.log gpurun_out/ab_g20.log | grep variant
