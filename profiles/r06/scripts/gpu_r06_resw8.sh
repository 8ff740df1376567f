#!/bin/bash
# round 6: resident v2 128x32 tiles with 8 waves (four column pairs per thread, LBM_RES_W8) vs the default 16 waves, 1024^2
set -o pipefail
OUT=gpurun_out/resw8
mkdir -p $OUT
timeout -k 10 300 python -u tools/ab_bench.py --n 1024 --steps 20000 --rounds 3 --check \
  --variant t:FLAGS=4,LBM_KERNEL=resident --variant t_w8:FLAGS=4,LBM_KERNEL=resident,LBM_RES_W8=1 2>&1 | tee $OUT/ab_tol.log &&
timeout -k 10 300 python -u tools/ab_bench.py --n 1024 --steps 20000 --rounds 3 --check \
  --variant b:LBM_KERNEL=resident --variant b_w8:LBM_KERNEL=resident,LBM_RES_W8=1 2>&1 | tee $OUT/ab_bit.log
