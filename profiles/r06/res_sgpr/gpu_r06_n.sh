#!/bin/bash
# Round 6, call N: resident v2 with the item coordinates opaque per step (the
# edge tests recomputed instead of hoisted as spilled SGPR lane masks) against
# the previous build (build_var/res_old), 1024^2 both numerics; the resident
# parity tests on the new build first.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
A="python3 tools/ab_bench.py --n 1024 --steps 2000 --warmup 200 --rounds 3 --variant b:LBM_RES_V=2 --variant t:LBM_RES_V=2,FLAGS=4"
bash tools/gpu_steps.sh \
  "600|pytest_res|python -u -m pytest tests/test_gpu_parity.py -k 'resident or division or signed_zero' tests/test_gpu_resident_recovery.py tests/test_gpu_tolerance.py -m gpu -x -q --timeout 200 --timeout-method thread" \
  "200|res_new_r1|$A" "200|res_old_r1|LBM_HIP_LIB=build_var/res_old/liblbm_hip.so $A" \
  "200|res_new_r2|$A" "200|res_old_r2|LBM_HIP_LIB=build_var/res_old/liblbm_hip.so $A" \
  "200|res_new_r3|$A" "200|res_old_r3|LBM_HIP_LIB=build_var/res_old/liblbm_hip.so $A" || exit $?
tail -n 1 gpurun_out/pytest_res.log; for f in gpurun_out/res_*_r*.log; do grep -h ms_median $f | sed "s#^#$f #" | cut -c1-150; done
