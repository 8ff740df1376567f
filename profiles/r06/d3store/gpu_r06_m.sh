#!/bin/bash
# Round 6, call M: the D3Q19 three-step pass with plain lattice stores (the
# new default) -- the 3-D GPU tests, the 512^3 bench in both numerics, and
# its kernel trace and PMC passes (FETCH_SIZE, WRITE_SIZE, SQ).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
D3="python3 tools/bench3d.py --n 512 --steps 12 --warmup 0 --flags 4"
bash tools/gpu_steps.sh \
  "600|pytest_d3|python -u -m pytest tests/test_d3q19.py tests/test_gpu_fullsize.py -k 'd3q19' -m gpu -x -q --timeout 200 --timeout-method thread" \
  "150|b3_f4|python3 tools/bench3d.py --n 512 --steps 60 --warmup 6 --rounds 3 --flags 4" \
  "150|b3_f0|python3 tools/bench3d.py --n 512 --steps 60 --warmup 6 --rounds 3 --flags 0" \
  "200|d3_trace|rocprofv3 --kernel-trace --stats -d gpurun_out/d3_trace -o d3 --output-format csv -- python3 tools/bench3d.py --n 512 --steps 30 --flags 4" \
  "150|d3_fetch|timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/d3_fetch -o fetch --output-format csv -- $D3" \
  "150|d3_write|timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/d3_write -o write --output-format csv -- $D3" \
  "150|d3_sq|timeout -s KILL 140 rocprofv3 --pmc $SQ -d gpurun_out/d3_sq -o sq --output-format csv -- $D3" || exit $?
tail -n 1 gpurun_out/pytest_d3.log; tail -n 1 gpurun_out/b3_f4.log; tail -n 1 gpurun_out/b3_f0.log
