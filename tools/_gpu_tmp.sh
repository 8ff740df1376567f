#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "500|sweep|python tools/ab_bench.py --n 8192 --steps 400 --rounds 3 --variant s4: --variant s3:LBM_STREAM_S=3 --variant s4w3:LBM_STREAM_W=3 --variant s3w3:LBM_STREAM_S=3,LBM_STREAM_W=3 --variant s2:LBM_STREAM_S=2"
grep -h mlups gpurun_out/sweep.log
