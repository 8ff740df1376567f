#!/usr/bin/env python3
"""A/B the step kernel's tuning knobs in ONE process (interleaved rounds).

Each variant is a set of LBM_* environment knobs read by lbm_create_ex
(LBM_KERNEL, LBM_STREAM_S/_V/_HS, LBM_TILE2, LBM_LAYOUT, LBM_MAX_BLOCKS,
LBM_GRAPH_STEPS, LBM_TWO_STEP, LBM_FORCE_EXCHANGE, LBM_XOFF); every LBM_*
variable is cleared before each variant.  For every round,
every variant creates an engine on the same synthetic problem, warms up and
times `steps` steps with the library's device events.  Prints one JSON line
per variant with the median / min ms per step and GB/s (72 B per update).

  python tools/ab_bench.py --n 8192 --steps 100 --rounds 3 \
      --variant base: --variant one:LBM_TWO_STEP=0 --variant planar:LBM_LAYOUT=planar
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "lbm-graphcore_amd")]

from lbm_amd import io as lio  # noqa: E402
from lbm_amd import native  # noqa: E402
from bench import synthetic_obstacles  # noqa: E402


def parse_variant(s: str):
    name, _, rest = s.partition(":")
    env = {}
    last = None
    for kv in filter(None, rest.split(",")):
        if "=" not in kv and last is not None:  # a value that itself contains commas
            env[last] += "," + kv
            continue
        k, _, v = kv.partition("=")
        env[k] = v
        last = k
    return name, env


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--ny", type=int, default=0)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variant", action="append", default=[])
    ap.add_argument("--check", action="store_true", help="also compare each variant's lattice to the first")
    ap.add_argument("--maps", default="", help="write /proc/self/maps to this file at interpreter exit "
                    "(maps the PCs of a crash in the C exit handlers, which run after it)")
    a = ap.parse_args()
    if a.maps:
        import atexit
        import shutil
        atexit.register(shutil.copyfile, "/proc/self/maps", a.maps)
    nx, ny = a.n, a.ny or a.n
    p = lio.Params(nx, ny, a.steps, 10, 0.1, 0.005, 1.85)
    obst = synthetic_obstacles(nx, ny)
    variants = [parse_variant(v) for v in (a.variant or ["base:"])]
    times = {name: [] for name, _ in variants}
    ref = None
    for rnd in range(a.rounds):
        for name, env in variants:
            for k in [k for k in os.environ if k.startswith("LBM_")]:
                os.environ.pop(k, None)
            os.environ.update({k: v for k, v in env.items() if k.startswith("LBM")})
            os.environ["LBM_DEBUG_KNOBS"] = "1"  # the library reads its knobs only with this set
            flags = int(env.get("FLAGS", "0"))    # e.g. FLAGS=4: LBM_FLAG_TOLERANCE
            with native.Engine(p, obst, devices=[0], flags=flags) as e:
                e.init_equilibrium()
                e.run_steps(a.warmup, accelerate_first=True)
                e.run_steps(a.steps)
                times[name].append(e.last_run_seconds() / a.steps)
                if a.check and rnd == 0:
                    cells, _ = e.store(n_av=1)
                    if ref is None:
                        ref = cells
                    elif not (cells == ref).all():
                        print(json.dumps({"variant": name, "error": "lattice differs from first variant"}))
    for name, env in variants:
        ts = times[name]
        med = statistics.median(ts)
        print(json.dumps({"variant": name, "env": env, "grid": f"{nx}x{ny}", "ms_median": round(med * 1e3, 4),
                          "ms_min": round(min(ts) * 1e3, 4),
                          "gbs_median": round(72 * nx * ny / med / 1e9, 1),
                          "mlups_median": round(nx * ny / med / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
