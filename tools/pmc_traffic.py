#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes into per-launch HBM traffic.

Recipe (/opt/skills/guides/MI355X_MICROARCH.md, HBM section): FETCH_SIZE and
WRITE_SIZE are collected in separate passes (they do not fit one TCC pass);
both are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide
(16 B/lane) coalesced streaming read, so it is doubled.  The step kernel's
loads are 16 B/lane float4 streams except one exec-masked dword per wave and
plane at row/wave seams and the 4 B/lane obstacle mask, so the doubled figure
slightly over-counts those narrow reads (upper bound).

  python tools/pmc_traffic.py --fetch DIR/fetch_counter_collection.csv \
      --write DIR/write_counter_collection.csv --key 8192x8192/step2 --cells 67108864 \
      [--sq DIR/sq_counter_collection.csv] --out profiles/traffic.json

--sq adds the VALU side of the same kernel from the SQ pass (tools/gpu_round.sh):
VALU instructions per launch and the VALU pipe's busy fraction,
4 x SQ_ACTIVE_INST_VALU (quad-cycles, summed over waves) / (SIMDs x
GRBM_GUI_ACTIVE / 8 XCDs) -- at two waves per SIMD only one issues VALU at a
time, so this is the share of SIMD cycles the VALU pipe was taken.
"""
from __future__ import annotations

import argparse
import csv
import json
import statistics
from pathlib import Path


def per_launch(path: str, counter: str, kernel_substr: str):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and kernel_substr in r["Kernel_Name"]]
    if not vals:
        raise SystemExit(f"no {counter} rows for kernels matching {kernel_substr!r} in {path}")
    return statistics.median(vals), len(vals)


def per_dispatch(path: str, kernel_substr: str):
    """Counter sums per dispatch (a counter may have one row per dimension), median over dispatches."""
    by = {}
    for r in csv.DictReader(open(path)):
        if kernel_substr not in r["Kernel_Name"]:
            continue
        d = by.setdefault(r["Dispatch_Id"], {})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    if not by:
        raise SystemExit(f"no rows for kernels matching {kernel_substr!r} in {path}")
    keys = set().union(*by.values())
    return {k: statistics.median(d[k] for d in by.values() if k in d) for k in keys}, len(by)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", default="step_vec4")
    ap.add_argument("--key", required=True)
    ap.add_argument("--cells", type=int, required=True)
    ap.add_argument("--out", default="profiles/traffic.json")
    ap.add_argument("--sq", default=None, help="SQ pass csv (SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU, GRBM_GUI_ACTIVE)")
    ap.add_argument("--simds", type=int, default=1024, help="SIMDs of the device (256 CUs x 4)")
    ap.add_argument("--profile", default=None, help="where the csv files are committed (recorded in the entry)")
    ap.add_argument("--bytes-per-cell", type=float, default=72.0,
                    help="algorithmic bytes per cell and launch (72: D2Q9; 152: a D3Q19 pass)")
    ap.add_argument("--fetch-mult", type=float, default=2.0,
                    help="FETCH_SIZE multiplier: 2 for 16 B/lane streams (guide); otherwise calibrated "
                         "on a kernel of the same access width with a known byte count (--fetch-note)")
    ap.add_argument("--fetch-note", default="gfx950 wide-stream undercount")
    a = ap.parse_args()
    fetch_kib, nf = per_launch(a.fetch, "FETCH_SIZE", a.kernel)
    write_kib, nw = per_launch(a.write, "WRITE_SIZE", a.kernel)
    read_b = a.fetch_mult * fetch_kib * 1024
    write_b = write_kib * 1024
    alg = a.bytes_per_cell * a.cells
    entry = {
        "kernel": a.kernel, "launches_fetch": nf, "launches_write": nw,
        "fetch_size_kib_raw": fetch_kib, "write_size_kib_raw": write_kib,
        "hbm_read_bytes_per_launch": read_b, "hbm_write_bytes_per_launch": write_b,
        "hbm_bytes_per_launch": read_b + write_b,
        "algorithmic_bytes_per_launch": alg,
        "ratio_to_algorithmic": round((read_b + write_b) / alg, 4),
        "correction": f"FETCH_SIZE x{a.fetch_mult:g} ({a.fetch_note}), KiB x1024",
    }
    if a.sq:
        sq, nd = per_dispatch(a.sq, a.kernel)
        cycles = sq["GRBM_GUI_ACTIVE"] / 8
        entry["valu"] = {
            "instr_per_launch": int(sq["SQ_INSTS_VALU"]),
            "busy_frac": round(4 * sq["SQ_ACTIVE_INST_VALU"] / (a.simds * cycles), 4),
            "clock_ghz_pmc_pass": round(cycles / (statistics.median(
                int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(a.sq))
                if a.kernel in r["Kernel_Name"]) * 1e-9) / 1e9, 3),
            "dispatches": nd,
            "def": "4 x SQ_ACTIVE_INST_VALU / (SIMDs x GRBM_GUI_ACTIVE / 8)",
        }
    if a.profile:
        entry["profile"] = a.profile
    out = Path(a.out)
    d = json.loads(out.read_text()) if out.exists() else {}
    d[a.key] = entry
    out.write_text(json.dumps(d, indent=1) + "\n")
    print(json.dumps({a.key: entry}))


if __name__ == "__main__":
    main()
