cd "$GRAFT_REPO_ROOT" || exit 2
bash tools/gpu_steps.sh "500|d3spread|LBM_DEBUG_KNOBS=1 LBM_PLACEMENT_LOG=1 python3 tools/d3_spread.py --engines 5"
cat gpurun_out/d3spread.log | grep "engine\|probe"
