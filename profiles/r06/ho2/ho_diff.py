#!/usr/bin/env python3
"""HO debug: one S-step launch with and without the strip hand-off, where the lattices differ."""
import os, sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[3]
sys.path[:0] = [str(ROOT), str(ROOT / "lbm-graphcore_amd")]
from lbm_amd import io as lio, native
from bench import synthetic_obstacles
os.environ["LBM_DEBUG_KNOBS"] = "1"
n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
res = {}
for ho in (0, 1):
    os.environ["LBM_STREAM_HO"] = str(ho)
    p = lio.Params(n, n, steps, 10, 0.1, 0.005, 1.85)
    with native.Engine(p, synthetic_obstacles(n, n), flags=4, kernel=native.KERNEL_STREAM) as e:
        e.init_equilibrium()
        e.run_steps(steps, accelerate_first=True)
        cells, av = e.store(n_av=steps)
        res[ho] = np.asarray(cells).reshape(n, n, 9)
d = np.any(res[0] != res[1], axis=2)
ys, xs = np.nonzero(d)
print("cells differing", d.sum(), "of", n * n)
if len(xs):
    cols = np.unique(xs)
    print("columns", len(cols), cols[:80].tolist())
    rows = np.unique(ys)
    print("rows", len(rows), rows[:40].tolist(), rows[-10:].tolist())
    planes = np.nonzero(np.any(res[0] != res[1], axis=(0, 1)))[0]
    print("planes", planes.tolist())
    k = np.argmax(d.ravel())
    y, x = divmod(int(k), n)
    print("first", y, x, res[0][y, x].tolist(), res[1][y, x].tolist())
