#!/usr/bin/env python3
"""Per-GPU cost of the decomposed path on ONE GPU: the same weak-scaling tile
(8192^2 per part) as one sub-domain and as R x C sub-domains on device 0
(LOCAL transport: boundary/interior split, halo pack/unpack, device copies).
A rate close to the single-domain one means the multi-GPU bench loses little
per GPU to decomposition overheads; the remaining difference on a real
multi-GPU node is the RCCL transfer itself.

  python tools/ab_parts.py --tile 8192 --grids 1x1 1x2 2x2 --steps 100
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
from bench import synthetic_obstacles  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tile", type=int, default=8192)
    ap.add_argument("--grids", nargs="+", default=["1x1", "1x2", "2x2"])
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--fixed", action="store_true", help="keep the global grid tile x tile (strong split)")
    a = ap.parse_args()
    for g in a.grids:
        R, C = (int(v) for v in g.split("x"))
        nx, ny = (a.tile, a.tile) if a.fixed else (a.tile * C, a.tile * R)
        p = lio.Params(nx, ny, a.steps, 10, 0.1, 0.005, 1.85)
        obst = synthetic_obstacles(nx, ny)
        with native.Engine(p, obst, parts=R * C, grid=(R, C), devices=[0]) as e:
            e.init_equilibrium()
            e.run_steps(a.warmup, accelerate_first=True)
            e.run_steps(a.steps)
            secs = e.last_run_seconds()
            kern = e.kernel_in_use()
        mlups = nx * ny * a.steps / secs / 1e6
        print(json.dumps({"grid": g, "cells": nx * ny, "kernel": kern, "ms_per_step": round(secs / a.steps * 1e3, 4),
                          "mlups": round(mlups, 1), "mlups_per_part": round(mlups / (R * C), 1)}), flush=True)


if __name__ == "__main__":
    main()
