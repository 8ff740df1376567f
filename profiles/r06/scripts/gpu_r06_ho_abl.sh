#!/bin/bash
# round 6: barrier-free strip hand-off ablations (LBM_STREAM_HO_DBG: 1 no waits, 2 no ring traffic, 4 no row counters; 1-7 give wrong lattices, timing only)
set -o pipefail
OUT=gpurun_out/ho2
mkdir -p $OUT
timeout -k 10 400 python -u tools/ab_bench.py --n 8192 --steps 100 --rounds 3 \
  --variant t10:FLAGS=4 --variant ho:FLAGS=4,LBM_STREAM_HO=1 --variant ho_nowait:FLAGS=4,LBM_STREAM_HO=1,LBM_STREAM_HO_DBG=5 \
  --variant ho_bare:FLAGS=4,LBM_STREAM_HO=1,LBM_STREAM_HO_DBG=7 2>&1 | tee $OUT/ab_abl.log
