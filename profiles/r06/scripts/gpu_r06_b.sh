#!/bin/bash
# Round 6, call B: FETCH_SIZE / WRITE_SIZE of the S = 10 tolerance launch with
# and without the mirrored segment walk (one PMC counter set per run).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp LBM_DEBUG_KNOBS=1 LBM_RES_COOP=0
V="--variant t10:FLAGS=4 --variant t10m:FLAGS=4,LBM_STREAM_MIRROR=1"
bash tools/gpu_steps.sh \
  "120|pmc_fetch_m|timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_m -o fetch --output-format csv -- python3 tools/ab_bench.py --n 8192 --steps 42 --warmup 6 --rounds 1 $V" \
  "120|pmc_write_m|timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_m -o write --output-format csv -- python3 tools/ab_bench.py --n 8192 --steps 42 --warmup 6 --rounds 1 $V" || exit $?
ls -R gpurun_out/pmc_fetch_m | head
