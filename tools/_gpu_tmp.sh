#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
ALT=lbm-graphcore_amd/build/alt/liblbm_hip.so
bash tools/gpu_steps.sh \
  "200|cr8192a|python tools/ab_bench.py --n 8192 --steps 200 --rounds 3 --variant cr:" \
  "200|fast8192a|env LBM_HIP_LIB=$ALT python tools/ab_bench.py --n 8192 --steps 200 --rounds 3 --variant fast:" \
  "200|cr8192b|python tools/ab_bench.py --n 8192 --steps 200 --rounds 3 --variant cr:" \
  "200|fast8192b|env LBM_HIP_LIB=$ALT python tools/ab_bench.py --n 8192 --steps 200 --rounds 3 --variant fast:" \
  "200|cr1024|python tools/ab_bench.py --n 1024 --steps 2000 --rounds 3 --variant cr:" \
  "200|fast1024|env LBM_HIP_LIB=$ALT python tools/ab_bench.py --n 1024 --steps 2000 --rounds 3 --variant fast:" \
  "300|fast_tests|env LBM_HIP_LIB=$ALT python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread"
grep -h "mlups\|passed\|failed" gpurun_out/cr8192a.log gpurun_out/fast8192a.log gpurun_out/cr8192b.log gpurun_out/fast8192b.log gpurun_out/cr1024.log gpurun_out/fast1024.log gpurun_out/fast_tests.log
