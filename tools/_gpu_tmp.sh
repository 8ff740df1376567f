#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "300|res_tests|python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'resident'" \
  "200|ab256|python tools/ab_bench.py --n 256 --steps 4000 --rounds 3 --variant v2:LBM_KERNEL=resident --variant v4:LBM_KERNEL=resident,LBM_RES_V=4" \
  "200|ab1024|python tools/ab_bench.py --n 1024 --steps 2000 --rounds 3 --variant v2:LBM_KERNEL=resident --variant v4:LBM_KERNEL=resident,LBM_RES_V=4"
grep -h "passed\|trace\]\|mlups" gpurun_out/res_tests.log gpurun_out/ab1024.log gpurun_out/ab256.log
