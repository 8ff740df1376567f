#!/usr/bin/env python3
"""Host overhead of one short timed run (the driver's 20 steps) at 8192^2: the
wall time of run_steps around the library's device time, repeated."""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "lbm-graphcore_amd")]

import torch  # noqa: E402

from lbm_amd import io as lio  # noqa: E402
from lbm_amd import native  # noqa: E402
from bench import synthetic_obstacles  # noqa: E402


def main():
    n, steps = 8192, int(sys.argv[1]) if len(sys.argv) > 1 else 20
    p = lio.Params(n, n, steps, 10, 0.1, 0.005, 1.85)
    with native.Engine(p, synthetic_obstacles(n, n), devices=[0], flags=native.FLAG_TOLERANCE,
                       steps_per_launch=7) as e:
        e.init_equilibrium()
        e.run_steps(5, accelerate_first=True)
        e.run_steps(1400)
        for i in range(8):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e.run_steps(steps)
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            dev = e.last_run_seconds()
            print(json.dumps({"i": i, "wall_ms": round(wall * 1e3, 4), "dev_ms": round(dev * 1e3, 4),
                              "host_ms": round((wall - dev) * 1e3, 4)}), flush=True)


if __name__ == "__main__":
    main()
