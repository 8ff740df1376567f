#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "400|pipe_tests|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cli.py -x -v --timeout 200 --timeout-method thread -k 'pipeline'" \
  "200|prof_pipe|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pipe -o pipe --output-format csv -- python3 bench.py --kernel pipeline --steps 50 --warmup 2 --no-cpu-baseline --no-aux"
cat gpurun_out/prof_pipe.log | grep metric
