"""Replay a sequence of D3Q19 engine configurations in one process and report
mismatches vs the oracle (debug aid for order-dependent failures)."""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "lbm-graphcore_amd"), str(ROOT / "tests")]
from lbm_amd import native  # noqa: E402
from oracle import oracle  # noqa: E402  (checker only)
import test_d3q19 as T  # noqa: E402

# ENVS[4] named the contiguous-allocation knob of an intermediate build (removed; now a no-op)
ENVS = [{}, {"LBM3D_KSPAD": "320"}, {"LBM3D_KSPAD": "64"}, {"LBM_LATTICE_PAD": "4096"},
        {"LBM_LATTICE_CONTIG": "1", "LBM3D_KSPAD": "64"}]
seq = sys.argv[1] if len(sys.argv) > 1 else "full"
cases = []
if seq == "full":
    for shape in ((64, 8, 5, 1), (70, 31, 24, 3)):
        for two in ("0", "1"):
            for i in range(5):
                cases.append((shape, two, i))
elif seq == "pair":  # two=0 then two=1, no knobs
    cases = [((70, 31, 24, 3), "0", 0), ((70, 31, 24, 3), "1", 0), ((70, 31, 24, 3), "1", 0)]
elif seq == "single_then":  # single-slab runs, then the slab case
    cases = [((64, 8, 5, 1), "1", 0)] * 6 + [((70, 31, 24, 3), "1", 0)] * 2
elif seq == "slab0_then":  # one-step slab runs, then the two-step slab case
    cases = [((70, 31, 24, 3), "0", 0)] * 6 + [((70, 31, 24, 3), "1", 0)] * 2
elif seq.startswith("knob"):  # knob run(s) env index N, then plain slab two-step runs
    ei = int(seq[4:])
    cases = [((70, 31, 24, 3), "1", ei)] * 2 + [((70, 31, 24, 3), "1", 0)] * 2 + [((64, 8, 5, 1), "1", ei)] * 2 + [((70, 31, 24, 3), "1", 0)] * 2
elif seq == "ones":
    cases = [((70, 31, 24, 3), "1", 0)] * 3
for (nx, ny, nz, parts), two, ei in cases:
    for k in [k for k in os.environ if k.startswith("LBM")]:
        os.environ.pop(k)
    os.environ.update(ENVS[ei])
    os.environ["LBM3D_TWO"] = two
    p, obst, c0 = T._problem(nx, ny, nz, nx + ny * nz)
    ref, _ = oracle.run3d(p, obst, 7, c0)
    cells, _ = T._gpu3d(native, p, obst, c0, 7, parts=parts, devices=[0])
    bad = np.argwhere(cells != ref)
    msg = ""
    if len(bad) and parts > 1:
        alt = {n: oracle.run3d(p, obst, n, c0)[0] for n in (5, 6, 8)}
        z0 = 0
        for i in range(parts):
            nzs = nz // parts + (1 if i < nz % parts else 0)
            sl = slice(z0, z0 + nzs)
            z0 += nzs
            eq = [n for n, r in alt.items() if np.array_equal(cells[sl], r[sl])]
            msg += f" slab{i}: {int((cells[sl] != ref[sl]).sum())} bad, equals steps {eq};"
    print(f"{seq}: {nx}x{ny}x{nz}/{parts} two={two} env={ENVS[ei]}: {len(bad)} bad{msg}", flush=True)
