#!/bin/bash
# round 6: barrier-free strip hand-off (LBM_STREAM_HO=1) -- lattice digests vs the default forms, then an interleaved A/B at 8192^2
set -o pipefail
OUT=gpurun_out/ho2
mkdir -p $OUT
export LBM_DEBUG_KNOBS=1
dig() { timeout -k 10 120 python -u tools/lattice_digest.py "$@"; }
{
for n in 2048 3000; do
  for st in 20 33 37 41; do
    for ho in 0 1; do
      LBM_STREAM_HO=$ho dig --n $n --steps $st --flags 4 | sed "s/^/ho=$ho /" || exit 1
    done
  done
done
for ho in 0 1; do LBM_TOL_S=8 LBM_STREAM_HO=$ho dig --n 2048 --steps 35 --flags 4 | sed "s/^/S8 ho=$ho /" || exit 1; done
for ho in 0 1; do LBM_TOL_S=6 LBM_STREAM_HO=$ho dig --n 2048 --steps 35 --flags 4 | sed "s/^/S6 ho=$ho /" || exit 1; done
} 2>&1 | tee $OUT/digests.log || exit 1
timeout -k 10 300 python -u tools/ab_bench.py --n 8192 --steps 100 --rounds 3 \
  --variant t10:FLAGS=4 --variant t10ho:FLAGS=4,LBM_STREAM_HO=1 2>&1 | tee $OUT/ab.log
