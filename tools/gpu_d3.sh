#!/bin/bash
# One GPU call for the D3Q19 row: its GPU tests, an interleaved A/B of the
# pass forms at 512^3, a kernel trace and the PMC passes (FETCH_SIZE,
# WRITE_SIZE, SQ counters -- each in its own run) of the default three-step
# pass in both numerics.  Logs under gpurun_out/d3/.
#   /usr/local/graft/bin/gpurun --timeout 1500 -- bash tools/gpu_d3.sh
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp LBM_DEBUG_KNOBS=1
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
AB='for r in 1 2 3; do for v in "tol:4:" "tol_noskip:4:LBM3D_SKIP3=0" "bw:0:" "bw_noskip:0:LBM3D_SKIP3=0" "bw_two:0:LBM3D_THREE=0"; do
  name=${v%%:*}; rest=${v#*:}; fl=${rest%%:*}; envs=${rest#*:}; echo -n "$name "; env $envs python3 tools/bench3d.py --n 512 --steps 30 --warmup 3 --flags $fl --rounds 2 || exit 1; done; done'
mkdir -p gpurun_out/d3
bash tools/gpu_steps.sh \
  "900|d3/pytest|python -u -m pytest tests/test_d3q19.py tests/test_gpu_fullsize.py tests/test_poison.py -m gpu -q -k 'd3q19 or D3 or 3d' --timeout 300 --timeout-method thread" \
  "600|d3/ab|$AB" \
  "200|d3/trace_tol|rocprofv3 --kernel-trace --stats -d gpurun_out/d3/trace_tol -o d3 --output-format csv -- python3 tools/bench3d.py --n 512 --steps 30 --flags 4" \
  "200|d3/trace_bw|rocprofv3 --kernel-trace --stats -d gpurun_out/d3/trace_bw -o d3 --output-format csv -- python3 tools/bench3d.py --n 512 --steps 30 --flags 0" \
  "150|d3/fetch_tol|timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/d3/fetch_tol -o fetch --output-format csv -- python3 tools/bench3d.py --n 512 --steps 12 --warmup 0 --flags 4" \
  "150|d3/write_tol|timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/d3/write_tol -o write --output-format csv -- python3 tools/bench3d.py --n 512 --steps 12 --warmup 0 --flags 4" \
  "150|d3/sq_tol|timeout -s KILL 140 rocprofv3 --pmc $SQ -d gpurun_out/d3/sq_tol -o sq --output-format csv -- python3 tools/bench3d.py --n 512 --steps 12 --warmup 0 --flags 4" \
  "150|d3/fetch_bw|timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/d3/fetch_bw -o fetch --output-format csv -- python3 tools/bench3d.py --n 512 --steps 12 --warmup 0 --flags 0" \
  "150|d3/write_bw|timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/d3/write_bw -o write --output-format csv -- python3 tools/bench3d.py --n 512 --steps 12 --warmup 0 --flags 0" \
  "150|d3/sq_bw|timeout -s KILL 140 rocprofv3 --pmc $SQ -d gpurun_out/d3/sq_bw -o sq --output-format csv -- python3 tools/bench3d.py --n 512 --steps 12 --warmup 0 --flags 0"
