# round 5: tolerance numerics after dropping the Newton step (every tolerance
# test, D3Q19 tolerance tests, resident tests), the driver's bench command, a
# kernel trace of it, and the PMC passes of the default S = 10 kernel.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
bash tools/gpu_steps.sh \
  "700|pytest_tol|python -u -m pytest tests/test_gpu_tolerance.py tests/test_d3q19.py tests/test_gpu_parity.py -k 'tolerance or resident' -q -s --timeout 300 --timeout-method thread; rc=\$?; [ \$rc -le 1 ]" \
  "400|bench_drv|python3 bench.py --gpus 1 --steps 20 --warmup 5" \
  "300|prof_trace|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o drv --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-aux" \
  "120|pmc_fetch|timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o fetch --output-format csv -- python3 tools/ab_bench.py --n 8192 --steps 60 --warmup 10 --rounds 1 --variant tol:FLAGS=4" \
  "120|pmc_write|timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o write --output-format csv -- python3 tools/ab_bench.py --n 8192 --steps 60 --warmup 10 --rounds 1 --variant tol:FLAGS=4" \
  "120|pmc_sq|timeout -s KILL 100 rocprofv3 --pmc $SQ -d gpurun_out/pmc_sq -o sq --output-format csv -- python3 tools/ab_bench.py --n 8192 --steps 60 --warmup 10 --rounds 1 --variant tol:FLAGS=4"
