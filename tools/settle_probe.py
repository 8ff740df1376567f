#!/usr/bin/env python3
"""Why does a short timed region (the driver's `--steps 20 --warmup 5`) run
slower per launch than a long one?  Mimics bench.py's setup, then times
back-to-back runs of `--steps` steps with the library's device events, once
right after the warm-up, then after an idle gap, printing one JSON line per
run.  A clock / power ramp shows up as slow first runs that speed up.

  python tools/settle_probe.py --n 8192 --steps 20 --warmup 5 --runs 12
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "lbm-graphcore_amd")]

from lbm_amd import io as lio  # noqa: E402
from lbm_amd import native  # noqa: E402
from bench import synthetic_obstacles  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--runs", type=int, default=12)
    ap.add_argument("--gap", type=float, default=1.0, help="idle seconds before the second series")
    a = ap.parse_args()
    p = lio.Params(a.n, a.n, a.steps, 10, 0.1, 0.005, 1.85)
    obst = synthetic_obstacles(a.n, a.n)
    with native.Engine(p, obst, devices=[0]) as e:
        e.init_equilibrium()
        e.run_steps(a.warmup, accelerate_first=True)
        spl = e.steps_per_launch()
        for series in ("after_warmup", "after_gap"):
            if series == "after_gap":
                time.sleep(a.gap)
            for r in range(a.runs):
                t = time.perf_counter()
                e.run_steps(a.steps)
                wall = time.perf_counter() - t
                dev = e.last_run_seconds()
                launches = max(a.steps // spl, 1)
                print(json.dumps({"series": series, "run": r, "dev_ms": round(dev * 1e3, 4),
                                  "ms_per_launch": round(dev / launches * 1e3, 4), "wall_ms": round(wall * 1e3, 3),
                                  "mlups": round(a.n * a.n * a.steps / dev / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
