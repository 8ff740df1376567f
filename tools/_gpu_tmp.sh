#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "300|stream_tests|python -m pytest tests/test_gpu_parity.py -q -x -k \"stream or open or large or reference\"" \
  "200|ab8192|python tools/ab_bench.py --n 8192 --steps 200 --rounds 3 --variant h48:LBM_STREAM_HS=48 --variant h64:LBM_STREAM_HS=64 --variant h96:LBM_STREAM_HS=96 --variant h128:LBM_STREAM_HS=128 --variant def: --variant s3:LBM_STREAM_S=3" \
  "200|ab4096|python tools/ab_bench.py --n 4096 --steps 400 --rounds 3 --variant def: --variant h32:LBM_STREAM_HS=32 --variant step2:LBM_KERNEL=step2" \
  "300|pmc_sq|rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU -d gpurun_out/pmc_sq3 -o sq --output-format csv -- python3 tools/ab_bench.py --n 8192 --steps 40 --warmup 4 --rounds 1 --variant v2:LBM_STREAM_HS=64"
