# round 5 verification on one box: the GPU suite, smoke, the driver's bench
# command and the default bench, a kernel trace of the driver command, and
# the PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) of the default S = 10 kernel.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
# PART: all (default), suite (GPU suite + smoke) or perf (the rest) -- a
# gpurun call is capped at 1200 s, so the two halves can go in separate calls
PART=${1:-all}
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
SUITE=("900|pytest_gpu|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread; rc=\$?; [ \$rc -le 1 ]" \
  "300|smoke|python -c 'import __graft_entry__ as g; g.smoke()'")
PERF=("400|bench_drv|python3 bench.py --gpus 1 --steps 20 --warmup 5" \
  "500|bench|python3 bench.py --no-cpu-baseline" \
  "300|prof_trace|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o drv --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-aux" \
  "120|pmc_fetch|timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o fetch --output-format csv -- python3 tools/ab_bench.py --n 8192 --steps 60 --warmup 10 --rounds 1 --variant tol:FLAGS=4" \
  "120|pmc_write|timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o write --output-format csv -- python3 tools/ab_bench.py --n 8192 --steps 60 --warmup 10 --rounds 1 --variant tol:FLAGS=4" \
  "120|pmc_sq|timeout -s KILL 100 rocprofv3 --pmc $SQ -d gpurun_out/pmc_sq -o sq --output-format csv -- python3 tools/ab_bench.py --n 8192 --steps 60 --warmup 10 --rounds 1 --variant tol:FLAGS=4")
case $PART in
  suite) bash tools/gpu_steps.sh "${SUITE[@]}" ;;
  perf) bash tools/gpu_steps.sh "${PERF[@]}" ;;
  *) bash tools/gpu_steps.sh "${SUITE[@]}" "${PERF[@]}" ;;
esac
rc=$?
[ "$PART" = perf ] || { grep -h "passed\|failed" gpurun_out/pytest_gpu.log | tail -3; tail -n 1 gpurun_out/smoke.log; }
exit $rc
