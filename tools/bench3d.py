#!/usr/bin/env python3
"""D3Q19 timing (BASELINE config 5): n^3 channel, one GPU or z slabs (loopback).

  python tools/bench3d.py --n 512 --steps 100 [--parts 1]
Prints one JSON line: MLUPS and the algorithmic HBM rate (152 B per update).
"""
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
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--parts", type=int, default=1)
    ap.add_argument("--flags", type=int, default=0, help="lbm_config flags (4 = LBM_FLAG_TOLERANCE)")
    ap.add_argument("--rounds", type=int, default=1, help="timed runs (the best is reported)")
    a = ap.parse_args()
    n = a.n
    p = lio.Params3D(n, n, n, a.steps, 0.1, 0.001, 1.85)
    with native.Engine3D(p, lio.channel_obstacles3d(n, n, n), parts=a.parts, devices=[0], flags=a.flags) as e:
        e.init_equilibrium()
        e.run_steps(a.warmup)
        secs = 1e30
        for _ in range(a.rounds):
            e.run_steps(a.steps)
            secs = min(secs, e.last_run_seconds())
    cells = n ** 3
    env = {k: v for k, v in __import__("os").environ.items() if k.startswith("LBM3D_")}
    print(json.dumps({"grid": f"{n}^3", "parts": a.parts, "steps": a.steps, "flags": a.flags, "env": env, "ms_per_step": round(secs / a.steps * 1e3, 4),
                      "mlups": round(cells * a.steps / secs / 1e6, 1),
                      "gbs": round(152 * cells * a.steps / secs / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
