#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "300|dec_tests|python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'decomp or exchange or stream or 16384'" \
  "500|strong|python tools/ab_parts.py --tile 16384 --fixed --grids 1x1 1x2 2x1 2x2 4x1 2x4 --steps 40" \
  "500|weak|python tools/ab_parts.py --tile 8192 --grids 1x1 1x2 2x1 2x2 4x1 --steps 100"
grep -h "passed\|failed" gpurun_out/dec_tests.log; grep -h mlups gpurun_out/strong.log gpurun_out/weak.log
