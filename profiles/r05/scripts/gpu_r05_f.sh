# round 5: wave timeline of the default S = 10 launch (slot efficiency, tail)
# and segment-tier (guide) variants at S = 10 in one process, interleaved.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp LBM_DEBUG_KNOBS=1
V="--variant g144:FLAGS=4 --variant g192:FLAGS=4,LBM_STREAM_GUIDE=192:0.85,64:0.1,16 --variant g240:FLAGS=4,LBM_STREAM_GUIDE=240:0.8,64:0.12,16 --variant g288:FLAGS=4,LBM_STREAM_GUIDE=288:0.75,96:0.15,24 --variant g144_8:FLAGS=4,LBM_STREAM_GUIDE=144:0.85,48:0.1,16:0.03,8 --variant g176:FLAGS=4,LBM_STREAM_GUIDE=176:0.8,56:0.12,16"
bash tools/gpu_steps.sh \
  "200|trace10|python3 tools/stream_trace.py --n 8192 --steps 60 --flags 4" \
  "500|ab_guide|python3 tools/ab_bench.py --n 8192 --steps 100 --warmup 10 --rounds 3 $V" \
  "300|ab_guide20|python3 tools/ab_bench.py --n 8192 --steps 20 --warmup 5 --rounds 5 $V"
rc=$?
grep variant gpurun_out/ab_guide.log gpurun_out/ab_guide20.log; cat gpurun_out/trace10.log | tail -2
exit $rc
