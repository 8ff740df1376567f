#!/bin/bash
# Round 6 verification of the final library on one box.  PART (a gpurun call
# is capped at 1200 s, so the halves go in separate calls):
#   suite -- the GPU suite and smoke;
#   perf  -- the driver's bench command (twice) and the default bench, a
#            rocprofv3 kernel trace of the driver command, the PMC passes
#            (FETCH_SIZE, WRITE_SIZE, SQ; each its own run) of the default
#            S = 10 stream launch at 8192^2, the D3Q19 512^3 three-step pass
#            (kernel trace, FETCH_SIZE, WRITE_SIZE, SQ) and the one-step D3Q19
#            kernel's FETCH_SIZE / WRITE_SIZE (calibration of the 4-B-per-lane
#            read width on a known byte count).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
PART=${1:-perf}
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
AB="python3 tools/ab_bench.py --n 8192 --steps 42 --warmup 6 --rounds 1 --variant tol:FLAGS=4"
D3="python3 tools/bench3d.py --n 512 --steps 12 --warmup 0 --flags 4"
D1="python3 tools/bench3d.py --n 512 --steps 4 --warmup 0 --flags 4"
SUITE=("900|pytest_gpu|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread; rc=\$?; [ \$rc -le 1 ]"
       "300|smoke|python -c 'import __graft_entry__ as g; g.smoke()'")
PERF=("300|bench_drv|python3 bench.py --gpus 1 --steps 20 --warmup 5"
      "300|bench_drv2|python3 bench.py --gpus 1 --steps 20 --warmup 5"
      "400|bench|python3 bench.py --no-cpu-baseline"
      "300|prof_trace|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o drv --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-aux"
      "120|pmc_fetch|timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o fetch --output-format csv -- $AB"
      "120|pmc_write|timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o write --output-format csv -- $AB"
      "120|pmc_sq|timeout -s KILL 100 rocprofv3 --pmc $SQ -d gpurun_out/pmc_sq -o sq --output-format csv -- $AB"
      "200|d3_trace|rocprofv3 --kernel-trace --stats -d gpurun_out/d3_trace -o d3 --output-format csv -- python3 tools/bench3d.py --n 512 --steps 30 --flags 4"
      "150|d3_fetch|timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/d3_fetch -o fetch --output-format csv -- $D3"
      "150|d3_write|timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/d3_write -o write --output-format csv -- $D3"
      "150|d3_sq|timeout -s KILL 140 rocprofv3 --pmc $SQ -d gpurun_out/d3_sq -o sq --output-format csv -- $D3"
      "150|d1_fetch|LBM_DEBUG_KNOBS=1 LBM3D_TWO=0 LBM3D_PAIR=0 timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/d1_fetch -o fetch --output-format csv -- $D1"
      "150|d1_write|LBM_DEBUG_KNOBS=1 LBM3D_TWO=0 LBM3D_PAIR=0 timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/d1_write -o write --output-format csv -- $D1")
case $PART in
  suite) bash tools/gpu_steps.sh "${SUITE[@]}" ;;
  *) bash tools/gpu_steps.sh "${PERF[@]}" ;;
esac
rc=$?
[ "$PART" = suite ] && { grep -h "passed\|failed" gpurun_out/pytest_gpu.log | tail -3; tail -n 1 gpurun_out/smoke.log; }
exit $rc
