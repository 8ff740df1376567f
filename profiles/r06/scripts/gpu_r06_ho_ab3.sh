#!/bin/bash
# round 6: HO vs the default form in four-wave workgroups (LBM_STREAM_W4, A/B only) vs the default
set -o pipefail
OUT=gpurun_out/ho2
mkdir -p $OUT
export LBM_DEBUG_KNOBS=1
{ for v in 0 1; do LBM_STREAM_HO=$v timeout -k 10 120 python -u tools/lattice_digest.py --n 3000 --steps 40 --flags 4 | sed "s/^/ho=$v /" || exit 1; done; } 2>&1 | tee $OUT/digests4.log || exit 1
timeout -k 10 300 python -u tools/ab_bench.py --n 8192 --steps 100 --rounds 3 \
  --variant t10:FLAGS=4 --variant ho:FLAGS=4,LBM_STREAM_HO=1 2>&1 | tee $OUT/ab4.log
