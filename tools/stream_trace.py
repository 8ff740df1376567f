#!/usr/bin/env python3
"""Wave timeline of one stream-kernel launch (diagnostics).

Runs the 8192^2 bench problem with LBM_STREAM_TRACE set, so the library dumps
{start, end} s_memrealtime stamps (100 MHz) of every wave of the last
interior launch, then prints: launch span, wave-duration spread, the share of
the device's wave slots kept busy (sum of wave durations / (slots x span)),
the busy-slot profile over time, and per-XCD first start / last end.

  LBM_DEBUG_KNOBS=1 python tools/stream_trace.py --n 8192 --slots 2048
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "lbm-graphcore_amd")]

from lbm_amd import io as lio  # noqa: E402
from lbm_amd import native  # noqa: E402
from bench import synthetic_obstacles  # noqa: E402


def analyse(tr: np.ndarray, slots: int, bins: int = 24) -> dict:
    st, en = tr[:, 0].astype(np.int64), tr[:, 1].astype(np.int64)
    ok = en > 0
    st, en = st[ok], en[ok]
    t0 = st.min()
    st, en = (st - t0) * 10e-3, (en - t0) * 10e-3  # microseconds
    span = float(en.max())
    dur = en - st
    edges = np.linspace(0, span, bins + 1)
    busy = []
    for a, b in zip(edges[:-1], edges[1:]):
        ov = np.clip(np.minimum(en, b) - np.maximum(st, a), 0, None).sum()
        busy.append(round(float(ov / (b - a) / slots), 3))
    xcd = np.arange(len(tr))[ok] & 7
    per_xcd = {int(x): [round(float(st[xcd == x].min()), 1), round(float(en[xcd == x].max()), 1)] for x in range(8)}
    return {"waves": int(ok.sum()), "span_us": round(span, 1),
            "dur_us": {"mean": round(float(dur.mean()), 1), "p10": round(float(np.percentile(dur, 10)), 1),
                       "p50": round(float(np.percentile(dur, 50)), 1), "p90": round(float(np.percentile(dur, 90)), 1),
                       "max": round(float(dur.max()), 1)},
            "slot_efficiency": round(float(dur.sum() / (slots * span)), 3),
            "busy_profile": busy, "xcd_first_start_last_end_us": per_xcd}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--slots", type=int, default=2048, help="resident waves the device holds (2/SIMD x 1024)")
    ap.add_argument("--flags", type=int, default=0, help="lbm_config flags (4 = LBM_FLAG_TOLERANCE: S = 7)")
    a = ap.parse_args()
    p = lio.Params(a.n, a.n, a.steps, 10, 0.1, 0.005, 1.85)
    obst = synthetic_obstacles(a.n, a.n)
    with tempfile.TemporaryDirectory() as wd:
        path = os.path.join(wd, "trace.bin")
        os.environ["LBM_STREAM_TRACE"] = path
        with native.Engine(p, obst, devices=[0], flags=a.flags) as e:
            e.init_equilibrium()
            e.run_steps(16, accelerate_first=True)
            e.run_steps(a.steps)
            ms = e.last_run_seconds() / max(a.steps // e.steps_per_launch(), 1) * 1e3
        tr = np.fromfile(path, dtype=np.uint64).reshape(-1, 2)
    out = analyse(tr, a.slots)
    out["ms_per_launch_events"] = round(ms, 4)
    out["flags"] = a.flags
    out["env"] = {k: v for k, v in os.environ.items() if k.startswith("LBM_") and k != "LBM_STREAM_TRACE"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
