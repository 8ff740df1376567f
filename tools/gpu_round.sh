#!/bin/bash
# One GPU call: tests, bench, A/B at 1024^2, rocprof kernel trace of the bench,
# and the two PMC passes for HBM traffic of the default kernel.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
A1024="--variant step2:LBM_KERNEL=step2 --variant s4:LBM_KERNEL=stream,LBM_STREAM_S=4 --variant s4h8:LBM_KERNEL=stream,LBM_STREAM_S=4,LBM_STREAM_HS=8 --variant s4h32:LBM_KERNEL=stream,LBM_STREAM_S=4,LBM_STREAM_HS=32 --variant s3:LBM_KERNEL=stream,LBM_STREAM_S=3 --variant s2:LBM_KERNEL=stream,LBM_STREAM_S=2 --variant v1s4:LBM_KERNEL=stream,LBM_STREAM_S=4,LBM_STREAM_V=1"
bash tools/gpu_steps.sh \
  "900|pytest_gpu|python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
  "400|bench|python bench.py" \
  "300|ab1024|python tools/ab_bench.py --n 1024 --steps 2000 --rounds 3 $A1024" \
  "300|prof_trace|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o bench --output-format csv -- python3 bench.py --steps 400 --no-cpu-baseline --no-aux" \
  "300|pmc_fetch|rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o fetch --output-format csv -- python3 tools/ab_bench.py --n 8192 --steps 40 --warmup 4 --rounds 1" \
  "300|pmc_write|rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o write --output-format csv -- python3 tools/ab_bench.py --n 8192 --steps 40 --warmup 4 --rounds 1"
