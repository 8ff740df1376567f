#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "500|hs|python tools/ab_bench.py --n 8192 --steps 500 --rounds 5 --variant auto: --variant h35:LBM_STREAM_HS=35 --variant h69:LBM_STREAM_HS=69 --variant h70:LBM_STREAM_HS=70"
grep -h mlups gpurun_out/hs.log
