#!/bin/bash
# round 6: segment tiers for the bitwise (VALU-bound) forms at 8192^2 -- taller tiers recompute fewer rows
set -o pipefail
OUT=gpurun_out/bwtiers
mkdir -p $OUT
timeout -k 10 600 python -u tools/ab_bench.py --n 8192 --steps 60 --rounds 3 \
  --variant b6:LBM_STREAM_S=6 \
  --variant b6_144:LBM_STREAM_S=6,LBM_STREAM_GUIDE=144:0.85,48:0.1,16 \
  --variant b6_192:LBM_STREAM_S=6,LBM_STREAM_GUIDE=192:0.85,64:0.1,16 \
  --variant b6_128:LBM_STREAM_S=6,LBM_STREAM_GUIDE=128:0.85,32:0.1,12 \
  --variant b5:LBM_STREAM_S=5 \
  --variant b5_144:LBM_STREAM_S=5,LBM_STREAM_GUIDE=144:0.85,48:0.1,16 \
  --variant b5_192:LBM_STREAM_S=5,LBM_STREAM_GUIDE=192:0.85,64:0.1,16 2>&1 | tee $OUT/ab_bw_tiers.log
