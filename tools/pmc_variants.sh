#!/bin/bash
# PMC passes (each its own run, per MI355X_MICROARCH.md) for tuning variants of
# the 8192^2 step kernel: SQ issue/stall counters + GRBM clock, FETCH_SIZE,
# WRITE_SIZE.  Summarise with tools/pmc_summary.py.
#   bash tools/pmc_variants.sh NAME "ENV=V ENV2=V2" [NAME2 "ENV..."] ...   (values without spaces)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
# ab_bench clears LBM_* itself and applies the variant's env (comma-separated)
while [ $# -ge 2 ]; do
  name="$1"; envs="$2"; shift 2
  for pass in sq fetch write; do
    case $pass in
      sq) ctr="$SQ" ;;
      fetch) ctr="FETCH_SIZE" ;;
      write) ctr="WRITE_SIZE" ;;
    esac
    out="gpurun_out/pmc/$name/$pass"
    mkdir -p "$out"
    echo "=== $name $pass ($envs)"
    timeout -s KILL 90 rocprofv3 --pmc $ctr -d "$out" -o run --output-format csv -- \
      python3 tools/ab_bench.py --n 8192 --steps 40 --warmup 8 --rounds 1 --variant "$name:${envs// /,}" > "$out/log.txt" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "pass $name/$pass failed rc=$rc"; tail -5 "$out/log.txt"; exit $rc; fi
  done
done
echo "=== pmc passes done"
