#!/bin/bash
# Round 6, call I: the one-step (vec4) and two-step (step2) kernels built
# without the SLP vectorizer (build_var/k_noslp, build_var/s2_noslp) against
# the default build, 8192^2 and 1024^2, one process per library interleaved;
# then the D3Q19 ablations (gpu_r06_h.sh).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
STEPS=()
for r in 1 2; do
  for n in 8192 1024; do
    A="python3 tools/ab_bench.py --n $n --steps 40 --warmup 6 --rounds 3"
    STEPS+=("150|k_def_${n}_r${r}|$A --variant vec4:LBM_KERNEL=vec4"
            "150|k_var_${n}_r${r}|LBM_HIP_LIB=build_var/k_noslp/liblbm_hip.so $A --variant vec4:LBM_KERNEL=vec4"
            "150|s2_def_${n}_r${r}|$A --variant step2:LBM_KERNEL=step2"
            "150|s2_var_${n}_r${r}|LBM_HIP_LIB=build_var/s2_noslp/liblbm_hip.so $A --variant step2:LBM_KERNEL=step2")
  done
done
bash tools/gpu_steps.sh "${STEPS[@]}" || exit $?
for f in gpurun_out/k_*_r*.log gpurun_out/s2_*_r*.log; do echo "$f $(grep ms_median $f | cut -c1-120)"; done
bash profiles/r06/scripts/gpu_r06_h.sh
