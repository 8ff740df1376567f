#!/usr/bin/env python3
"""Engine-to-engine spread of the D3Q19 two-step pass at n^3:
creates `--engines` engines one after another in one process, times `--steps`
steps on each (best of `--rounds`), prints one JSON line per engine."""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "lbm-graphcore_amd")]

from lbm_amd import io as lio  # noqa: E402
from lbm_amd import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--engines", type=int, default=6)
    ap.add_argument("--flags", type=int, default=0)
    a = ap.parse_args()
    n = a.n
    p = lio.Params3D(n, n, n, a.steps, 0.1, 0.001, 1.85)
    obst = lio.channel_obstacles3d(n, n, n)
    for i in range(a.engines):
        with native.Engine3D(p, obst, devices=[0], flags=a.flags) as e:
            e.init_equilibrium()
            e.run_steps(6)
            best = 1e30
            for _ in range(a.rounds):
                e.run_steps(a.steps)
                best = min(best, e.last_run_seconds())
        print(json.dumps({"engine": i, "grid": f"{n}^3", "ms_per_step": round(best / a.steps * 1e3, 4),
                          "mlups": round(n ** 3 * a.steps / best / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
