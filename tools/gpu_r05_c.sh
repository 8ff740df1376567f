# round 5: A/B of the stream-kernel revisions as libraries (one process per
# library, interleaved), the LP-form parity tests, and the exit-time crash
# experiment under rocprofv3 (the crashing configuration last).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
AB="python3 tools/ab_bench.py --n 8192 --steps 100 --warmup 10 --rounds 2 --variant t10:FLAGS=4 --variant b6:LBM_STREAM_S=6 --variant b5:LBM_STREAM_S=5"
bash tools/gpu_steps.sh \
  "300|ab_new1|$AB" \
  "300|ab_old1|LBM_HIP_LIB=build_var/r04stream/liblbm_hip.so $AB" \
  "300|ab_nn1|LBM_HIP_LIB=build_var/nonewton/liblbm_hip.so $AB" \
  "300|ab_new2|$AB" \
  "300|ab_old2|LBM_HIP_LIB=build_var/r04stream/liblbm_hip.so $AB" \
  "300|ab_nn2|LBM_HIP_LIB=build_var/nonewton/liblbm_hip.so $AB" \
  "400|pytest_c|python -u -m pytest tests/test_gpu_cli.py tests/test_gpu_bench.py tests/test_gpu_tolerance.py::test_tolerance_steps_per_launch_invariant tests/test_gpu_tolerance.py::test_tolerance_8192_vs_oracle tests/test_gpu_parity.py -k 'cli or bench or invariant or 8192 or stream6 or plain6 or size_limits' -q --timeout 300 --timeout-method thread; rc=\$?; [ \$rc -le 1 ]" \
  "200|exit_stream|mkdir -p gpurun_out/exit_stream && rocprofv3 --kernel-trace --stats -d gpurun_out/exit_stream -o s --output-format csv -- python3 tools/ab_bench.py --n 1024 --steps 20000 --warmup 200 --rounds 1 --variant s:FLAGS=4,LBM_KERNEL=stream" \
  "200|exit_plain|mkdir -p gpurun_out/exit_plain && rocprofv3 --kernel-trace --stats -d gpurun_out/exit_plain -o v2 --output-format csv -- python3 tools/ab_bench.py --n 1024 --steps 20000 --warmup 200 --rounds 1 --variant t:FLAGS=4,LBM_RES_V=2,LBM_RES_COOP=0"
rc=$?
for f in ab_new1 ab_old1 ab_nn1 ab_new2 ab_old2 ab_nn2; do echo "== $f"; grep variant gpurun_out/$f.log; done
exit $rc
