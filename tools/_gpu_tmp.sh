#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
: > gpurun_out/d3_ab.log
for r in 1 2; do
  for cfg in "0 32" "1 32" "1 64" "1 128" "1 256"; do
    set -- $cfg
    echo "two=$1 seg=$2 round=$r $(env LBM3D_TWO=$1 LBM3D_SEG=$2 timeout -k 10 120 python tools/bench3d.py --n 512 --steps 40 | tail -n 1)" >> gpurun_out/d3_ab.log || exit 1
  done
done
cat gpurun_out/d3_ab.log
