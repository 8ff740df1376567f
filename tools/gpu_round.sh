#!/bin/bash
# One GPU call (gpurun): the round's verification -- GPU tests, smoke, the
# driver's exact bench command and the default bench, a rocprofv3 kernel trace
# of the driver's command, and the PMC passes (FETCH_SIZE, WRITE_SIZE and the
# SQ counters, each in its own run) of the default kernel at 8192^2.
#   /usr/local/graft/bin/gpurun --timeout 1500 -- bash tools/gpu_round.sh
# then: python3 tools/pmc_traffic.py --fetch gpurun_out/pmc_fetch/fetch_counter_collection.csv \
#         --write gpurun_out/pmc_write/write_counter_collection.csv --kernel "stream_steps2d<7" \
#         --sq gpurun_out/pmc_sq/sq_counter_collection.csv --key 8192x8192/stream7t --cells 67108864 \
#         --profile "profiles/rNN/...: kernel, date" --out profiles/traffic.json
# The pytest step continues on test FAILURES (exit 1: the rest still runs, the
# log says what failed) but stops on anything else (crash, abort, timeout).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
bash tools/gpu_steps.sh \
  "900|pytest_gpu|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread; rc=\$?; [ \$rc -le 1 ]" \
  "300|smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "400|bench_drv|python3 bench.py --gpus 1 --steps 20 --warmup 5" \
  "500|bench|python3 bench.py --no-cpu-baseline" \
  "300|prof_trace|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o drv --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-aux" \
  "120|pmc_fetch|timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o fetch --output-format csv -- python3 tools/ab_bench.py --n 8192 --steps 42 --warmup 6 --rounds 1 --variant tol:FLAGS=4" \
  "120|pmc_write|timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o write --output-format csv -- python3 tools/ab_bench.py --n 8192 --steps 42 --warmup 6 --rounds 1 --variant tol:FLAGS=4" \
  "120|pmc_sq|timeout -s KILL 100 rocprofv3 --pmc $SQ -d gpurun_out/pmc_sq -o sq --output-format csv -- python3 tools/ab_bench.py --n 8192 --steps 42 --warmup 6 --rounds 1 --variant tol:FLAGS=4" \
  "200|d3_trace|rocprofv3 --kernel-trace --stats -d gpurun_out/d3_trace -o d3 --output-format csv -- python3 tools/bench3d.py --n 512 --steps 30 --flags 4" \
  "150|d3_fetch|timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/d3_fetch -o fetch --output-format csv -- python3 tools/bench3d.py --n 512 --steps 12 --warmup 0 --flags 4" \
  "150|d3_write|timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/d3_write -o write --output-format csv -- python3 tools/bench3d.py --n 512 --steps 12 --warmup 0 --flags 4"
grep -h "passed\|failed" gpurun_out/pytest_gpu.log; tail -n 2 gpurun_out/smoke.log; tail -n 1 gpurun_out/bench.log
