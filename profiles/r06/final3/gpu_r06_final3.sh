#!/bin/bash
# Round 6 close: the committed library (sources unchanged since final2; rebuilt after the HO experiment was removed): the GPU suite,
# smoke, the driver's bench command twice, the default bench and a rocprofv3
# kernel trace of the driver command (the 2-D kernels are unchanged since
# gpu_r06_final.sh, whose PMC passes stand).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "900|pytest_gpu|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread; rc=\$?; [ \$rc -le 1 ]" \
  "300|smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "300|bench_drv|python3 bench.py --gpus 1 --steps 20 --warmup 5" \
  "300|bench_drv2|python3 bench.py --gpus 1 --steps 20 --warmup 5" \
  "300|prof_trace|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o drv --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-aux" || exit $?
grep -h "passed\|failed" gpurun_out/pytest_gpu.log | tail -2; tail -n 1 gpurun_out/smoke.log
