#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "400|d3q19_tests|python -u -m pytest tests/test_d3q19.py -x -q --timeout 200 --timeout-method thread" \
  "200|prof3d|rocprofv3 --kernel-trace --stats -d gpurun_out/prof3d -o d3 --output-format csv -- python3 tools/bench3d.py --n 512 --steps 30"
