#!/bin/bash
# v5 (two-cell ring resident kernel) vs v2 at 1024^2, with the timing-only
# breakdown builds (tools/build_variant.sh r5v8 "-DR5_DBG=8" lbm_resident2:
# no poll; r5v40 "-DR5_DBG=40": no poll, no publish) and kernel traces of both.
# Run on the GPU box from the repo root; writes gpurun_out/res5/.
set -e
mkdir -p gpurun_out/res5
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/ab_bench.py --n 1024 --steps 20000 --warmup 200 --rounds 3 \
  --variant v2_tol:FLAGS=4,LBM_RES_V=2 --variant v5_tol:FLAGS=4,LBM_RES_V=5 \
  --variant v2_bitwise:LBM_RES_V=2 --variant v5_bitwise:LBM_RES_V=5 > gpurun_out/res5/ab.log 2>&1
for v in r5v8 r5v40; do
  echo "== $v" >> gpurun_out/res5/ab.log
  LBM_HIP_LIB=build_var/$v/liblbm_hip.so timeout -k 10 120 python3 tools/ab_bench.py --n 1024 --steps 20000 \
    --warmup 200 --rounds 2 --variant v5_tol:FLAGS=4,LBM_RES_V=5 >> gpurun_out/res5/ab.log 2>&1
done
for v in 2 5; do
  LBM_DEBUG_KNOBS=1 LBM_RES_V=$v timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/res5/trace_v$v -o v$v --output-format csv -- \
    python3 tools/ab_bench.py --n 1024 --steps 20000 --warmup 200 --rounds 1 --variant t:FLAGS=4,LBM_RES_V=$v > gpurun_out/res5/trace_v$v.log 2>&1
done
cat gpurun_out/res5/ab.log
