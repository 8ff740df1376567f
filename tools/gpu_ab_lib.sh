# A/B of the default build against one variant library (tools/build_variant.sh):
#   bash tools/gpu_ab_lib.sh TAG build_var/NAME/liblbm_hip.so [pairs]
# GPU parity of the default build (stream kernel files), lattice digests of
# both builds, then one process per library interleaved `pairs` times;
# logs gpurun_out/TAG_*.log.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp LBM_DEBUG_KNOBS=1
TAG=$1 LIB=$2 N=${3:-3}
V="--variant t10:FLAGS=4 --variant t8:FLAGS=4,LBM_TOL_S=8 --variant b5: --variant b6:LBM_STREAM_S=6"
AB="python3 tools/ab_bench.py --n 8192 --steps 100 --warmup 10 --rounds 3 $V"
D="python3 tools/lattice_digest.py --n 2048 --steps 33"
STEPS=("600|${TAG}_parity|python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_tolerance.py tests/test_gpu_ordering.py tests/test_poison.py"
       "200|${TAG}_dig|for f in 4 0; do $D --flags \$f; LBM_HIP_LIB=$LIB $D --flags \$f; done")
for i in $(seq 1 "$N"); do
  STEPS+=("200|${TAG}_def$i|$AB" "200|${TAG}_var$i|LBM_HIP_LIB=$LIB $AB")
done
bash tools/gpu_steps.sh "${STEPS[@]}" || exit $?
cat "gpurun_out/${TAG}_dig.log"
python3 - "$TAG" "$N" <<'PY'
import json, sys, statistics
tag, n = sys.argv[1], int(sys.argv[2])
res = {}
for side in ("def", "var"):
    for i in range(1, n + 1):
        for line in open(f"gpurun_out/{tag}_{side}{i}.log"):
            if line.startswith("{"):
                d = json.loads(line)
                res.setdefault((d["variant"], side), []).append(d["ms_median"])
for v in sorted({k[0] for k in res}):
    a, b = res[(v, "def")], res[(v, "var")]
    print(f"{v}: default {statistics.median(a):.4f} {a}  variant {statistics.median(b):.4f} {b}  "
          f"variant/default {statistics.median(b) / statistics.median(a):.3f}")
PY
