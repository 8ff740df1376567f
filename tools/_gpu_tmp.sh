#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
ALT=lbm-graphcore_amd/build/alt/liblbm_hip.so
bash tools/gpu_steps.sh \
  "300|stream_tests|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cli.py -x -q --timeout 120 --timeout-method thread -k 'stream or auto or 8192 or exchange or decomp'" \
  "200|new8192a|python tools/ab_bench.py --n 8192 --steps 200 --rounds 3 --variant buf:" \
  "200|old8192a|env LBM_HIP_LIB=$ALT python tools/ab_bench.py --n 8192 --steps 200 --rounds 3 --variant old:" \
  "200|new8192b|python tools/ab_bench.py --n 8192 --steps 200 --rounds 3 --variant buf:" \
  "200|old8192b|env LBM_HIP_LIB=$ALT python tools/ab_bench.py --n 8192 --steps 200 --rounds 3 --variant old:" \
  "200|new4096|python tools/ab_bench.py --n 4096 --steps 400 --rounds 3 --variant buf:" \
  "200|old4096|env LBM_HIP_LIB=$ALT python tools/ab_bench.py --n 4096 --steps 400 --rounds 3 --variant old:"
grep -h "mlups\|passed\|failed" gpurun_out/stream_tests.log gpurun_out/new8192a.log gpurun_out/old8192a.log gpurun_out/new8192b.log gpurun_out/old8192b.log gpurun_out/new4096.log gpurun_out/old4096.log
