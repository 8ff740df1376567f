# round 5: A/B of the stage-interleaved tolerance collision (build_var/ilv,
# LBM_EXP_ILV=1) against the default library, one process per library,
# interleaved; plus its bitwise identity with the default on one problem.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
AB="python3 tools/ab_bench.py --n 8192 --steps 100 --warmup 10 --rounds 2 --variant t10:FLAGS=4 --variant t8:FLAGS=4,LBM_TOL_S=8 --variant t6:FLAGS=4,LBM_TOL_S=6"
bash tools/gpu_steps.sh \
  "300|ab_def1|$AB" \
  "300|ab_ilv1|LBM_HIP_LIB=build_var/ilv/liblbm_hip.so $AB" \
  "300|ab_def2|$AB" \
  "300|ab_ilv2|LBM_HIP_LIB=build_var/ilv/liblbm_hip.so $AB" \
  "300|same|python3 tools/lattice_digest.py --n 2048 --steps 33 --flags 4 > gpurun_out/dig_def.txt && LBM_HIP_LIB=build_var/ilv/liblbm_hip.so python3 tools/lattice_digest.py --n 2048 --steps 33 --flags 4 > gpurun_out/dig_ilv.txt && cat gpurun_out/dig_def.txt gpurun_out/dig_ilv.txt && cmp gpurun_out/dig_def.txt gpurun_out/dig_ilv.txt"
rc=$?
for f in ab_def1 ab_ilv1 ab_def2 ab_ilv2; do echo "== $f"; grep variant gpurun_out/$f.log; done
exit $rc
