"""Debug helper: v5 resident kernel vs the oracle, repeated runs (races show
as run-to-run differences); prints failing-run counts per configuration."""
import os, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "lbm-graphcore_amd")]
os.environ["LBM_DEBUG_KNOBS"] = "1"
os.environ["LBM_RES_V"] = os.environ.get("RESV", "5")
import numpy as np
from lbm_amd import io as lio
from lbm_amd import native
from oracle import oracle

tag = os.environ.get("LBM_HIP_LIB", "default")
for (nx, ny, steps, reps, tol) in [(128, 32, 2, 20, 0), (128, 32, 6, 10, 0), (256, 64, 6, 6, 0), (128, 32, 6, 10, 1)]:
    p = lio.Params(nx, ny, steps, 10, 0.1, 0.02, 1.7)
    obst = np.zeros((ny, nx), np.uint8)
    rng = np.random.default_rng(1)
    cells0 = (lio.init_cells(p) * (1 + 0.05 * rng.standard_normal((ny, nx, 9)))).astype(np.float32)
    ref, _ = oracle.run(p, obst, steps, cells0)
    fails, cellsets, outs = 0, set(), []
    for r in range(reps):
        with native.Engine(p, obst, kernel=native.KERNEL_RESIDENT, flags=native.FLAG_TOLERANCE if tol else 0) as e:
            e.load_cells(cells0)
            e.run_steps(steps, accelerate_first=True)
            cells, _ = e.store(n_av=1)
        if tol:
            outs.append(cells)
            continue
        bad = np.argwhere(cells != ref)
        if len(bad):
            fails += 1
            cellsets |= set(map(tuple, bad[:, :2].tolist()))
    if tol:
        fails = sum(not np.array_equal(o, outs[0]) for o in outs[1:])
    print(f"[{tag}] {nx}x{ny} steps={steps} tol={tol}: {fails}/{reps} runs differ; cells {sorted(cellsets)[:10]}", flush=True)
