# round 5: LP |u| sums in VGPRs (build_var/usumv, LBM_LP_USUM_LDS=0) against
# LDS (default build), one process per library, interleaved four times.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp LBM_DEBUG_KNOBS=1
NEW=build_var/usumv/liblbm_hip.so
V="--variant t10:FLAGS=4 --variant b6:LBM_STREAM_S=6"
AB="python3 tools/ab_bench.py --n 8192 --steps 100 --warmup 10 --rounds 3 $V"
bash tools/gpu_steps.sh \
  "200|us2_def1|$AB" "200|us2_v1|LBM_HIP_LIB=$NEW $AB" \
  "200|us2_def2|$AB" "200|us2_v2|LBM_HIP_LIB=$NEW $AB" \
  "200|us2_def3|$AB" "200|us2_v3|LBM_HIP_LIB=$NEW $AB" \
  "200|us2_def4|$AB" "200|us2_v4|LBM_HIP_LIB=$NEW $AB" || exit $?
for f in def1 v1 def2 v2 def3 v3 def4 v4; do echo "# $f"; grep variant gpurun_out/us2_$f.log; done
