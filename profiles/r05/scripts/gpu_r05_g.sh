# round 5 (g): stream-kernel parity after the in-place shifts and register
# |u| sums, lattice digests (must equal profiles/r05/swap/sw_dig_*), the
# driver's bench command.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "600|g_parity|python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_tolerance.py tests/test_gpu_ordering.py tests/test_gpu_bench.py" \
  "120|g_dig|for f in 4 0; do python3 tools/lattice_digest.py --n 2048 --steps 33 --flags \$f; done" \
  "300|g_bench|python3 bench.py --steps 20 --warmup 5" || exit $?
cat gpurun_out/g_dig.log; tail -1 gpurun_out/g_bench.log | cut -c1-400
