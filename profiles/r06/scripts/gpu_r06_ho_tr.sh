#!/bin/bash
# round 6: HO wave timelines and work split vs the default form (8192^2 tolerance)
set -o pipefail
OUT=gpurun_out/ho2
mkdir -p $OUT
export LBM_DEBUG_KNOBS=1 LBM_STREAM_DEBUG=1
{ timeout -k 10 120 python -u tools/stream_trace.py --n 8192 --steps 60 --flags 4 &&
  LBM_STREAM_HO=1 timeout -k 10 120 python -u tools/stream_trace.py --n 8192 --steps 60 --flags 4; } 2>&1 | tee $OUT/trace.log
