#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "300|big|python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k test_16384_lattice_64bit_indexing" \
  "300|stream_tests|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cli.py -x -q --timeout 120 --timeout-method thread -k 'stream or auto or 8192 or exchange or decomp or vec4 or scalar'" \
  "300|ab16384|python tools/ab_bench.py --n 16384 --steps 40 --rounds 1 --variant s4:"
grep -h "passed\|failed" gpurun_out/big.log gpurun_out/stream_tests.log; grep -h mlups gpurun_out/ab16384.log
