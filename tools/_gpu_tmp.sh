#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "300|pf_tests|LBM_STREAM_PF=2 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k 'stream or large or open'" \
  "300|ab_pf|python tools/ab_bench.py --n 8192 --steps 200 --rounds 4 --variant pf1:LBM_STREAM_PF=1 --variant pf2:LBM_STREAM_PF=2 && python tools/ab_bench.py --n 4096 --steps 400 --rounds 3 --variant pf1:LBM_STREAM_PF=1 --variant pf2:LBM_STREAM_PF=2"
