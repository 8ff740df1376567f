# round 5: x-shifted planes kept swapped (in-place DPP shifts, LBM_SWAP_SHIFT)
# against the in-order build (build_var/noswap): stream parity tests, lattice
# digests of both builds, and an interleaved one-process-per-library A/B.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp LBM_DEBUG_KNOBS=1
OLD=build_var/noswap/liblbm_hip.so
V="--variant t10:FLAGS=4 --variant t8:FLAGS=4,LBM_TOL_S=8 --variant b5: --variant b6:LBM_STREAM_S=6"
AB="python3 tools/ab_bench.py --n 8192 --steps 100 --warmup 10 --rounds 2 $V"
bash tools/gpu_steps.sh \
  "400|sw_parity|python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_tolerance.py -k 'stream or tolerance or Stream'" \
  "120|sw_dig_new|for f in 4 0; do python3 tools/lattice_digest.py --n 2048 --steps 33 --flags \$f; done" \
  "120|sw_dig_old|for f in 4 0; do LBM_HIP_LIB=$OLD python3 tools/lattice_digest.py --n 2048 --steps 33 --flags \$f; done" \
  "300|sw_ab_new1|$AB" \
  "300|sw_ab_old1|LBM_HIP_LIB=$OLD $AB" \
  "300|sw_ab_new2|$AB" \
  "300|sw_ab_old2|LBM_HIP_LIB=$OLD $AB" || exit $?
cat gpurun_out/sw_dig_new.log gpurun_out/sw_dig_old.log
for f in new1 old1 new2 old2; do echo "# $f"; grep variant gpurun_out/sw_ab_$f.log; done
