#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "300|res_tests|python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'resident'" \
  "200|trace|python tools/ab_bench.py --n 1024 --steps 300 --rounds 1 --variant v2:LBM_KERNEL=resident,LBM_RES_TRACE=1 --variant v1:LBM_KERNEL=resident,LBM_RES_TRACE=1,LBM_RES_V=1 && python tools/ab_bench.py --n 128 --steps 300 --rounds 1 --variant v2:LBM_KERNEL=resident,LBM_RES_TRACE=1 --variant v1:LBM_KERNEL=resident,LBM_RES_TRACE=1,LBM_RES_V=1" \
  "200|ab1024|python tools/ab_bench.py --n 1024 --steps 2000 --rounds 3 --variant step2:LBM_KERNEL=step2 --variant v1:LBM_KERNEL=resident,LBM_RES_V=1 --variant v2:LBM_KERNEL=resident,LBM_RES_V=2" \
  "200|ab256|python tools/ab_bench.py --n 256 --steps 4000 --rounds 3 --variant step2:LBM_KERNEL=step2 --variant v1:LBM_KERNEL=resident,LBM_RES_V=1 --variant r2:LBM_KERNEL=resident,LBM_RES_TH=2 --variant r4:LBM_KERNEL=resident,LBM_RES_TH=4,LBM_RES_V=2 --variant v1r8:LBM_KERNEL=resident,LBM_RES_TH=8,LBM_RES_V=1" \
  "200|ab128|python tools/ab_bench.py --n 128 --steps 4000 --rounds 3 --variant step2:LBM_KERNEL=step2 --variant v1:LBM_KERNEL=resident,LBM_RES_V=1 --variant r2:LBM_KERNEL=resident,LBM_RES_TH=2 --variant r4:LBM_KERNEL=resident,LBM_RES_TH=4,LBM_RES_V=2"
grep -h "trace\|mlups" gpurun_out/trace.log gpurun_out/ab*.log
