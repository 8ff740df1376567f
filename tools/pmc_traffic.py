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
      --out profiles/traffic.json
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", default="step_vec4")
    ap.add_argument("--key", required=True)
    ap.add_argument("--cells", type=int, required=True)
    ap.add_argument("--out", default="profiles/traffic.json")
    a = ap.parse_args()
    fetch_kib, nf = per_launch(a.fetch, "FETCH_SIZE", a.kernel)
    write_kib, nw = per_launch(a.write, "WRITE_SIZE", a.kernel)
    read_b = 2.0 * fetch_kib * 1024
    write_b = write_kib * 1024
    alg = 72 * a.cells
    entry = {
        "kernel": a.kernel, "launches_fetch": nf, "launches_write": nw,
        "fetch_size_kib_raw": fetch_kib, "write_size_kib_raw": write_kib,
        "hbm_read_bytes_per_launch": read_b, "hbm_write_bytes_per_launch": write_b,
        "hbm_bytes_per_launch": read_b + write_b,
        "algorithmic_bytes_per_launch": alg,
        "ratio_to_algorithmic": round((read_b + write_b) / alg, 4),
        "correction": "FETCH_SIZE x2 (gfx950 wide-stream undercount), KiB x1024",
    }
    out = Path(a.out)
    d = json.loads(out.read_text()) if out.exists() else {}
    d[a.key] = entry
    out.write_text(json.dumps(d, indent=1) + "\n")
    print(json.dumps({a.key: entry}))


if __name__ == "__main__":
    main()
