#!/usr/bin/env python3
"""Summarise tools/pmc_variants.sh output: per variant, per dispatch of the
step kernel (median over dispatches): duration, effective clock
(GRBM_GUI_ACTIVE / 8 XCDs / duration), SQ issue and stall counters (quad
cycles, summed over waves), VALU instructions, and HBM bytes (FETCH_SIZE x 2
per the gfx950 note, WRITE_SIZE) against the algorithmic 72 B x cells.

  python tools/pmc_summary.py gpurun_out/pmc --kernel stream_steps --cells 67108864
"""
from __future__ import annotations

import argparse
import csv
import json
import statistics
from collections import defaultdict
from pathlib import Path


def load(path: Path, kernel: str):
    by_disp = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if kernel not in r["Kernel_Name"]:
            continue
        d = by_disp[r["Dispatch_Id"]]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        d["_dur_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        d["_kernel"] = r["Kernel_Name"][:60]
    return list(by_disp.values())


def med(rows, key):
    vals = [r[key] for r in rows if key in r]
    return statistics.median(vals) if vals else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--kernel", default="stream_steps")
    ap.add_argument("--cells", type=int, default=8192 * 8192)
    a = ap.parse_args()
    for vdir in sorted(Path(a.root).iterdir()):
        out = {"variant": vdir.name}
        for pass_ in ("sq", "fetch", "write"):
            files = list((vdir / pass_).glob("**/*counter_collection.csv"))
            if not files:
                continue
            rows = load(files[0], a.kernel)
            if not rows:
                continue
            out.setdefault("kernel", rows[0]["_kernel"])
            dur = med(rows, "_dur_ns")
            out[f"dur_us_{pass_}"] = round(dur / 1e3, 1)
            if pass_ == "sq":
                for k in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY",
                          "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_INSTS_SALU", "GRBM_GUI_ACTIVE"):
                    v = med(rows, k)
                    if v is not None:
                        out[k] = v
                if "GRBM_GUI_ACTIVE" in out:
                    clk = out["GRBM_GUI_ACTIVE"] / 8 / (dur * 1e-9)
                    out["clock_ghz"] = round(clk / 1e9, 3)
                    simd_cycles = 1024 * out["GRBM_GUI_ACTIVE"] / 8
                    if "SQ_INSTS_VALU" in out:
                        out["valu_instr_per_simd_cycle"] = round(out["SQ_INSTS_VALU"] / simd_cycles, 4)
                wc = out.get("SQ_WAVE_CYCLES")
                if wc:
                    for k in ("SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"):
                        if k in out:
                            out[k + "_frac"] = round(out[k] / wc, 3)
            elif pass_ == "fetch":
                out["hbm_read_GB"] = round(2 * med(rows, "FETCH_SIZE") * 1024 / 1e9, 3)
            else:
                out["hbm_write_GB"] = round(med(rows, "WRITE_SIZE") * 1024 / 1e9, 3)
        if "hbm_read_GB" in out and "hbm_write_GB" in out:
            tot = out["hbm_read_GB"] + out["hbm_write_GB"]
            out["hbm_GB"] = round(tot, 3)
            out["ratio_to_algorithmic"] = round(tot * 1e9 / (72 * a.cells), 4)
            out["read_ratio"] = round(out["hbm_read_GB"] * 1e9 / (36 * a.cells), 4)
            if "dur_us_fetch" in out:
                out["hbm_TBps_fetchpass"] = round(tot * 1e9 / (out["dur_us_fetch"] * 1e-6) / 1e12, 3)
        print(json.dumps(out))


if __name__ == "__main__":
    main()
