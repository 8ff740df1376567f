#!/bin/bash
# Round 6, call F: D3Q19 three-step pass restructured (register sets per plane
# parity, static row liveness, buffer addressing) against the round-6 no-SLP build (build_var/old3d) -- the 3-D GPU tests on
# the new default, then an interleaved A/B of both libraries at 512^3 in both
# numerics.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
B="python3 tools/bench3d.py --n 512 --steps 60 --warmup 6 --rounds 2"
STEPS=("600|pytest_d3|python -u -m pytest tests/test_d3q19.py -m gpu -x -q --timeout 120 --timeout-method thread"
       "300|pytest_d3_full|python -u -m pytest tests/test_gpu_fullsize.py -k d3q19 -x -q --timeout 200 --timeout-method thread")
for r in 1 2; do
  for f in 4 0; do
    STEPS+=("150|ab_new_f${f}_r${r}|$B --flags $f" "150|ab_old_f${f}_r${r}|LBM_HIP_LIB=build_var/old3d/liblbm_hip.so $B --flags $f")
  done
done
bash tools/gpu_steps.sh "${STEPS[@]}" || exit $?
for f in gpurun_out/ab_*_f*.log; do echo "$f $(tail -n 1 $f | cut -c1-160)"; done
