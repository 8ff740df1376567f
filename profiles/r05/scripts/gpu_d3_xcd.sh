# D3Q19 passes with the XCD-aware block order (default build) against the
# hardware order (build_var/d3hw, LBM3D_XCD_REMAP=0): D3Q19 GPU tests of the
# default build, then one process per library interleaved, and the FETCH_SIZE
# pass of each (tolerance, three-step).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp LBM_DEBUG_KNOBS=1
OLD=build_var/d3hw/liblbm_hip.so
B="python3 tools/bench3d.py --n 512 --steps 30 --warmup 3 --rounds 2"
AB='for r in 1 2 3; do for lib in new old; do for fl in 4 0; do
  if [ $lib = old ]; then L=LBM_HIP_LIB='$OLD'; else L=; fi; echo -n "$lib fl$fl "; env $L '"$B"' --flags $fl || exit 1; done; done; done'
mkdir -p gpurun_out/d3x
bash tools/gpu_steps.sh \
  "600|d3x/pytest|python -u -m pytest tests/test_d3q19.py tests/test_gpu_ordering.py -m gpu -q -k 'd3q19 or 3d' --timeout 300 --timeout-method thread" \
  "600|d3x/ab|$AB" \
  "150|d3x/fetch_new|timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/d3x/fetch_new -o fetch --output-format csv -- python3 tools/bench3d.py --n 512 --steps 12 --warmup 0 --flags 4" \
  "150|d3x/fetch_old|LBM_HIP_LIB=$OLD timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/d3x/fetch_old -o fetch --output-format csv -- python3 tools/bench3d.py --n 512 --steps 12 --warmup 0 --flags 4" || exit $?
cat gpurun_out/d3x/ab.log | cut -c1-200
