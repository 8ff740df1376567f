#!/bin/bash
# Round 6, call J: resident kernel v6 (register rows + edge waves, opt-in
# LBM_RES_V=6) -- its GPU parity tests, then an A/B against v2 at 1024^2
# (BASELINE config 2) in both numerics, and one traced run of each.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
A="python3 tools/ab_bench.py --n 1024 --steps 2000 --warmup 200 --rounds 3"
V="--variant v2b:LBM_RES_V=2 --variant v6b:LBM_RES_V=6 --variant v2t:LBM_RES_V=2,FLAGS=4 --variant v6t:LBM_RES_V=6,FLAGS=4"
bash tools/gpu_steps.sh \
  "300|pytest_v6|python -u -m pytest tests/test_gpu_resident_v6.py -x -v --timeout 120 --timeout-method thread" \
  "200|ab_v6_r1|$A $V" \
  "200|ab_v6_r2|$A $V" \
  "200|trace_v6|python3 tools/ab_bench.py --n 1024 --steps 300 --warmup 50 --rounds 1 --variant v6t:LBM_RES_V=6,FLAGS=4,LBM_RES_TRACE=1 --variant v2t:LBM_RES_V=2,FLAGS=4,LBM_RES_TRACE=1" || exit $?
grep -h ms_median gpurun_out/ab_v6_r*.log | cut -c1-150; grep -h "resident trace" gpurun_out/trace_v6.log | head -4
