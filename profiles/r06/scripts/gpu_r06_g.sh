#!/bin/bash
# Round 6, call G: D3Q19 three-step pass, three builds interleaved at 512^3 in
# both numerics -- the default (restructured: register sets per plane parity,
# static row liveness, buffer addressing, input planes two deep), pd1 (the
# same with one plane in flight) and old3d (the round-6 no-SLP kernel before
# the restructure); the 3-D GPU tests on the default first (argument "ab":
# the A/B only).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
B="python3 tools/bench3d.py --n 512 --steps 60 --warmup 6 --rounds 2"
STEPS=()
[ "$1" = ab ] || STEPS=("600|pytest_d3|python -u -m pytest tests/test_d3q19.py -m gpu -x -q --timeout 120 --timeout-method thread"
       "300|pytest_d3_full|python -u -m pytest tests/test_gpu_fullsize.py -k d3q19 -x -q --timeout 200 --timeout-method thread")
for r in 1 2 3; do
  for f in 4 0; do
    STEPS+=("150|ab_pd2_f${f}_r${r}|$B --flags $f"
            "150|ab_pd1_f${f}_r${r}|LBM_HIP_LIB=build_var/pd1/liblbm_hip.so $B --flags $f"
            "150|ab_old_f${f}_r${r}|LBM_HIP_LIB=build_var/old3d/liblbm_hip.so $B --flags $f")
  done
done
bash tools/gpu_steps.sh "${STEPS[@]}" || exit $?
for f in gpurun_out/ab_*_f*_r*.log; do echo "$f $(tail -n 1 $f | cut -c60-130)"; done
