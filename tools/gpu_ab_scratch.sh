cd "$GRAFT_REPO_ROOT" || exit 2
export LBM_DEBUG_KNOBS=1
B="python3 tools/bench3d.py --n 512 --steps 60 --rounds 3"
bash tools/gpu_steps.sh \
  "500|ab_three|LBM3D_THREE=0 $B && LBM3D_THREE=1 $B && LBM3D_THREE=1 LBM3D_SEG3=128 $B && LBM3D_THREE=0 $B --flags 4 && LBM3D_THREE=1 $B --flags 4 && LBM3D_THREE=1 LBM3D_SEG3=128 $B --flags 4 && LBM3D_THREE=0 $B && LBM3D_THREE=1 $B && LBM3D_THREE=0 $B --flags 4 && LBM3D_THREE=1 $B --flags 4"
cat gpurun_out/ab_three.log | grep mlups
