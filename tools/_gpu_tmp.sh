#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "300|res_tests|LBM_RES_EARLY=1 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'resident'" \
  "200|hop|python tools/ab_bench.py --n 1024 --steps 200 --rounds 1 --variant e0:LBM_KERNEL=resident,LBM_RES_TRACE=2 --variant e1:LBM_KERNEL=resident,LBM_RES_TRACE=2,LBM_RES_EARLY=1 --variant v3:LBM_KERNEL=resident,LBM_RES_TRACE=2,LBM_RES_V=3" \
  "200|ab1024|python tools/ab_bench.py --n 1024 --steps 2000 --rounds 3 --variant e0:LBM_KERNEL=resident --variant e1:LBM_KERNEL=resident,LBM_RES_EARLY=1"
grep -h "hop\]\|mlups" gpurun_out/hop.log gpurun_out/ab1024.log
