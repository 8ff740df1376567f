#!/bin/bash
# Round 6, call C: D3Q19 three-step pass on 32 x 24 tiles (LBM3D_TW3=32, the
# new default) against 64 x 12 tiles -- the 3-D GPU tests, the 512^3 slab
# tests, an interleaved A/B of both tile shapes in both numerics, and the
# driver's 2-D bench command.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
AB=""
for r in 1 2; do
  for tw in 32 64; do
    for f in 4 0; do
      AB="$AB \"150|ab_tw${tw}_f${f}_r${r}|LBM_DEBUG_KNOBS=1 LBM3D_TW3=$tw python3 tools/bench3d.py --n 512 --steps 60 --warmup 6 --rounds 2 --flags $f\""
    done
  done
done
eval bash tools/gpu_steps.sh \
  "\"600|pytest_d3|python -u -m pytest tests/test_d3q19.py -m gpu -x -q --timeout 120 --timeout-method thread\"" \
  "\"300|pytest_d3_full|python -u -m pytest tests/test_gpu_fullsize.py -k d3q19 -x -q --timeout 200 --timeout-method thread\"" \
  $AB \
  "\"300|bench_drv|python3 bench.py --gpus 1 --steps 20 --warmup 5\"" || exit $?
for f in gpurun_out/ab_tw*.log; do echo "$f $(tail -n 1 $f | cut -c1-200)"; done
