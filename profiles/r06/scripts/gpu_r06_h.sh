#!/bin/bash
# Round 6, call H: ablations of the D3Q19 three-step pass at 512^3 (tolerance),
# timing-only builds of lbm3d.hip (results not meaningful): nocoll (the
# collision replaced by a pass-through), nobar (no level barriers), l2 (every
# load from the segment's first two planes: L2-resident), nost (no lattice
# stores) -- interleaved with the default build, two rounds.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
B="python3 tools/bench3d.py --n 512 --steps 60 --warmup 6 --rounds 2 --flags 4"
STEPS=()
for r in 1 2; do
  STEPS+=("150|abl_def_r${r}|$B")
  for v in nocoll nobar l2 nost; do
    STEPS+=("150|abl_${v}_r${r}|LBM_HIP_LIB=build_var/abl_${v}/liblbm_hip.so $B")
  done
done
bash tools/gpu_steps.sh "${STEPS[@]}" || exit $?
for f in gpurun_out/abl_*_r*.log; do echo "$f $(tail -n 1 $f | cut -c60-130)"; done
