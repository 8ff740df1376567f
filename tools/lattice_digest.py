#!/usr/bin/env python3
"""sha256 of the lattice after a run of the bench problem (synthetic obstacles,
equilibrium start) -- compares two library builds (LBM_HIP_LIB) for bitwise
identity without a CPU oracle run.

  python tools/lattice_digest.py --n 2048 --steps 33 --flags 4
"""
from __future__ import annotations

import argparse
import hashlib
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "lbm-graphcore_amd")]

from lbm_amd import io as lio  # noqa: E402
from lbm_amd import native  # noqa: E402
from bench import synthetic_obstacles  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=33)
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--spl", type=int, default=0)
    a = ap.parse_args()
    p = lio.Params(a.n, a.n, a.steps, 10, 0.1, 0.005, 1.85)
    with native.Engine(p, synthetic_obstacles(a.n, a.n), flags=a.flags, kernel=native.KERNEL_STREAM,
                       steps_per_launch=a.spl) as e:
        e.init_equilibrium()
        e.run_steps(a.steps, accelerate_first=True)
        cells, av = e.store(n_av=a.steps)
        print(f"{a.n}x{a.n} steps {a.steps} flags {a.flags} S {e.steps_per_launch()} "
              f"lattice {hashlib.sha256(cells.tobytes()).hexdigest()} av {hashlib.sha256(av.tobytes()).hexdigest()}")


if __name__ == "__main__":
    main()
