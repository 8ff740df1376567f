#!/bin/bash
# Round 6, call K: D3Q19 three-step pass, z planes per block (LBM3D_SEG3) at
# 512^3 tolerance and bitwise, two interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
STEPS=()
for r in 1 2; do
  for g in 64 32 128 256 512; do
    for f in 4 0; do
      STEPS+=("120|seg_${g}_f${f}_r${r}|LBM_DEBUG_KNOBS=1 LBM3D_SEG3=$g python3 tools/bench3d.py --n 512 --steps 60 --warmup 6 --rounds 2 --flags $f")
    done
  done
done
bash tools/gpu_steps.sh "${STEPS[@]}" || exit $?
for f in gpurun_out/seg_*.log; do echo "$f $(tail -n 1 $f | cut -c60-140)"; done
