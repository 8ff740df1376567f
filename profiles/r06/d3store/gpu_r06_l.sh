#!/bin/bash
# Round 6, call L: D3Q19 three-step pass with plain (temporal) lattice stores
# (build_var/st_plain) against the default non-temporal stores, 512^3, both
# numerics, three interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
B="python3 tools/bench3d.py --n 512 --steps 60 --warmup 6 --rounds 2"
STEPS=()
for r in 1 2 3; do
  for f in 4 0; do
    STEPS+=("120|st_nt_f${f}_r${r}|$B --flags $f" "120|st_plain_f${f}_r${r}|LBM_HIP_LIB=build_var/st_plain/liblbm_hip.so $B --flags $f")
  done
done
bash tools/gpu_steps.sh "${STEPS[@]}" || exit $?
for f in gpurun_out/st_*.log; do echo "$f $(tail -n 1 $f | cut -c60-140)"; done
