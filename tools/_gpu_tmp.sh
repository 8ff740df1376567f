#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "200|res16x8_test|LBM_RES_PER_CU=2 LBM_RES_TH=16 LBM_RES_V=2 python -u -m pytest 'tests/test_gpu_parity.py::test_resident_1024_runs_continue[2]' -x -q --timeout 120 --timeout-method thread" \
  "200|ab1024|python tools/ab_bench.py --n 1024 --steps 2000 --rounds 3 --variant v2:LBM_KERNEL=resident,LBM_RES_V=2 --variant v2x2:LBM_KERNEL=resident,LBM_RES_V=2,LBM_RES_PER_CU=2,LBM_RES_TH=16 --variant v2x2t:LBM_KERNEL=resident,LBM_RES_V=2,LBM_RES_PER_CU=2,LBM_RES_TH=16,LBM_RES_TRACE=1"
grep -h "trace\]\|mlups" gpurun_out/ab1024.log
