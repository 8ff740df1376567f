#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "300|res_tests|python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'resident'" \
  "200|trace|python tools/ab_bench.py --n 1024 --steps 300 --rounds 1 --variant v3:LBM_KERNEL=resident,LBM_RES_TRACE=1,LBM_RES_V=3 --variant v3b:LBM_KERNEL=resident,LBM_RES_TRACE=1,LBM_RES_V=3,LBM_RES_TH=32 && python tools/ab_bench.py --n 128 --steps 300 --rounds 1 --variant v3:LBM_KERNEL=resident,LBM_RES_TRACE=1,LBM_RES_V=3" \
  "200|ab1024|python tools/ab_bench.py --n 1024 --steps 2000 --rounds 3 --variant v2:LBM_KERNEL=resident,LBM_RES_V=2 --variant v3:LBM_KERNEL=resident,LBM_RES_V=3" \
  "200|ab256|python tools/ab_bench.py --n 256 --steps 4000 --rounds 3 --variant v2:LBM_KERNEL=resident,LBM_RES_V=2 --variant v3_4:LBM_KERNEL=resident,LBM_RES_V=3,LBM_RES_TH=4 --variant v3_2:LBM_KERNEL=resident,LBM_RES_V=3,LBM_RES_TH=2 --variant v3_8:LBM_KERNEL=resident,LBM_RES_V=3,LBM_RES_TH=8" \
  "200|ab128|python tools/ab_bench.py --n 128 --steps 4000 --rounds 3 --variant v2:LBM_KERNEL=resident,LBM_RES_V=2 --variant v3_4:LBM_KERNEL=resident,LBM_RES_V=3,LBM_RES_TH=4 --variant v3_2:LBM_KERNEL=resident,LBM_RES_V=3,LBM_RES_TH=2 --variant v3_8:LBM_KERNEL=resident,LBM_RES_V=3,LBM_RES_TH=8"
grep -h "trace\]\|mlups" gpurun_out/trace.log gpurun_out/ab*.log
