cd "$GRAFT_REPO_ROOT" || exit 2
G="--variant g96:FLAGS=4 --variant g128:FLAGS=4,LBM_STREAM_GUIDE=128:0.8,48:0.15,16 --variant g144:FLAGS=4,LBM_STREAM_GUIDE=144:0.85,48:0.1,16 --variant g192:FLAGS=4,LBM_STREAM_GUIDE=192:0.75,64:0.15,24 --variant g120:FLAGS=4,LBM_STREAM_GUIDE=120:0.9,40 --variant g112:FLAGS=4,LBM_STREAM_GUIDE=112:0.85,40:0.1,14"
bash tools/gpu_steps.sh \
  "400|ab_guide7|python3 tools/ab_bench.py --n 8192 --steps 98 --warmup 14 --rounds 3 $G" \
  "300|ab_guide7_20|python3 tools/ab_bench.py --n 8192 --steps 20 --warmup 5 --rounds 3 $G"
cat gpurun_out/ab_guide7.log gpurun_out/ab_guide7_20.log | grep variant
