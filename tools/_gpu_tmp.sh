#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_d3q19.py -x -q --timeout 240 --timeout-method thread -m gpu > gpurun_out/d3_tests.log 2>&1 || { tail -30 gpurun_out/d3_tests.log; exit 1; }
: > gpurun_out/d3_ab2.log
for r in 1 2; do
  for cfg in "0 64" "1 64" "1 128"; do
    set -- $cfg
    echo "two=$1 seg=$2 round=$r $(env LBM3D_TWO=$1 LBM3D_SEG=$2 timeout -k 10 120 python tools/bench3d.py --n 512 --steps 40 | tail -n 1)" >> gpurun_out/d3_ab2.log || exit 1
  done
done
tail -1 gpurun_out/d3_tests.log; cat gpurun_out/d3_ab2.log
