#!/bin/bash
# Round 6, call A: the whole GPU suite on the split engine + resident
# recovery, the mirrored-walk parity tests, then an interleaved A/B at 8192^2
# of the mirrored walk (LBM_STREAM_MIRROR) and of the refactored unit entry
# against the round-5 stream kernel source (build_var/old).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
V="--variant t10:FLAGS=4 --variant t10m:FLAGS=4,LBM_STREAM_MIRROR=1 --variant b6:LBM_STREAM_S=6 --variant b6m:LBM_STREAM_S=6,LBM_STREAM_MIRROR=1"
AB="env LBM_DEBUG_KNOBS=1 python3 tools/ab_bench.py --n 8192 --steps 100 --warmup 10 --rounds 3 $V"
OLD="env LBM_DEBUG_KNOBS=1 LBM_HIP_LIB=build_var/old/liblbm_hip.so python3 tools/ab_bench.py --n 8192 --steps 100 --warmup 10 --rounds 3 --variant t10:FLAGS=4 --variant b6:LBM_STREAM_S=6"
bash tools/gpu_steps.sh \
  "300|t_mirror|python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k mirrored" \
  "900|pytest_gpu|python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread; rc=\$?; [ \$rc -le 1 ]" \
  "200|ab1|$AB" "200|old1|$OLD" "200|ab2|$AB" "200|old2|$OLD" || exit $?
grep -h "passed\|failed" gpurun_out/pytest_gpu.log
grep -h variant gpurun_out/ab1.log gpurun_out/old1.log gpurun_out/ab2.log gpurun_out/old2.log
