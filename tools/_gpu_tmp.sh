#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "500|strong|python tools/ab_parts.py --tile 16384 --fixed --grids 1x1 1x2 2x1 2x2 4x1 2x4 8x1 --steps 40"
grep -h mlups gpurun_out/strong.log
