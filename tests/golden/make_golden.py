#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ (run in the build
container, where /root/reference exists; the GPU box only reads the output).

  check/*.dat.gz      the reference's own check/*.dat fixtures, gzipped (data)
  params/*            the reference's params/obstacles input files (data)
  oracle/<grid>.json  for each reference grid, from the CPU oracle restatement
                      (oracle/lbm_oracle.c) at the full step count:
                        sha256 of the final AoS float32 lattice (bitwise GPU gate),
                        free cells, Reynolds number, and -- when oracle/_ref exists --
                        whether the reference's own LastChance binary produced
                        byte-identical av_vels.dat / final_state.dat text
  oracle/<grid>.av_vels.npy.gz   oracle av_vels (float32) for every step
  oracle/<grid>.final_state_pressure.npy.gz
                      the pressure column of the oracle's final_state.dat
                      (float32[ny][nx], writeResults' arithmetic) -- the
                      second file of the check.py gate on the grids whose
                      check/*.final_state.dat the reference does not ship
                      (256x256, 1024x1024: /root/reference/.MISSING_LARGE_BLOBS);
                      the oracle's final_state text is byte-identical to the
                      reference binary's on every grid (oracle/<grid>.json)
  small.npz           full lattices after 1, 2 and 10 steps on small synthetic
                      problems (walls, interior wall, ragged widths, 1-row grid)
  oracle_pipe/<grid>.json, .av_vels.npy.gz
                      the same for the UNFUSED pipeline restatement
                      (oracle_pipe_run: accelerate every step, textbook BGK),
                      plus its check.py result against the reference fixtures

Usage: python tests/golden/make_golden.py [--grids 128x128,...] [--jobs N]
"""
from __future__ import annotations

import argparse
import gzip
import hashlib
import io as _io
import json
import os
import sys
import tempfile
from concurrent.futures import ProcessPoolExecutor
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "lbm-graphcore_amd"))

from oracle import oracle  # noqa: E402  (test infrastructure)
from lbm_amd import io as lio  # noqa: E402

GOLD = ROOT / "tests" / "golden"
GRIDS = ["128x128", "128x256", "256x256", "1024x1024"]


def lattice_sha256(cells: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(cells, dtype="<f4").tobytes()).hexdigest()


def grid_files(grid: str):
    return GOLD / "params" / f"input_{grid}.params", GOLD / "params" / f"obstacles_{grid}.dat"


def run_grid(grid: str) -> dict:
    pf, of = grid_files(grid)
    p = lio.Params.from_file(str(pf))
    obst = lio.read_obstacles(p.nx, p.ny, str(of))
    cells, av = oracle.run(p, obst)
    out = {
        "grid": grid, "nx": p.nx, "ny": p.ny, "steps": p.max_iters,
        "free_cells": oracle.free_cells(p, obst),
        "final_f_sha256": lattice_sha256(cells),
        "reynolds_last_av": oracle.reynolds(p, float(av[-1])),
        "reynolds_final_state": oracle.reynolds(p, oracle.av_velocity(p, cells, obst)),
        "total_density": float(np.sum(cells, dtype=np.float64)),
    }
    buf = _io.BytesIO()
    np.save(buf, av.astype(np.float32))
    (GOLD / "oracle" / f"{grid}.av_vels.npy.gz").write_bytes(gzip.compress(buf.getvalue(), 9))
    # pin against the reference binary itself when it was built here
    if oracle.REF_LASTCHANCE.exists():
        with tempfile.TemporaryDirectory() as wd:
            ref = oracle.run_reference(str(pf), str(of), wd)
            lio_av = os.path.join(wd, "ours_av.dat")
            with open(lio_av, "w") as f:  # LastChance's own printf format (LastChance.cpp:629)
                f.write("".join(f"{i}:\t{float(v):.12E}\n" for i, v in enumerate(av)))
            ref_av = open(ref["av_vels"]).read()
            ours_av = open(lio_av).read()
            ux, uy, u, pr = lio.macroscopic(p, obst, cells)
            lines = []
            for jj in range(p.ny):
                for ii in range(p.nx):
                    # LastChance.cpp:614 prints obstacles[ii*nx+jj] (transposed index)
                    t = ii * p.nx + jj
                    ob = int(obst.ravel()[t]) if t < obst.size else 0
                    lines.append(f"{ii} {jj} {ux[jj, ii]:.12E} {uy[jj, ii]:.12E} {u[jj, ii]:.12E} "
                                 f"{pr[jj, ii]:.12E} {ob}\n")
            ref_fs = open(ref["final_state"]).read().splitlines(keepends=True)
            # compare the numeric columns (the obstacle column is read out of bounds upstream)
            same_fs = all(a.rsplit(" ", 1)[0] == b.rsplit(" ", 1)[0] for a, b in zip(lines, ref_fs)) and \
                len(lines) == len(ref_fs)
            out["reference_binary"] = {
                "av_vels_identical": ref_av == ours_av,
                "final_state_identical": bool(same_fs),
                "reference_elapsed_s": ref.get("elapsed_s"),
                "reference_reynolds": ref.get("reynolds"),
            }
    (GOLD / "oracle" / f"{grid}.json").write_text(json.dumps(out, indent=1) + "\n")
    return out


def run_pipe_grid(grid: str) -> dict:
    from lbm_amd import check as lcheck
    pf, of = grid_files(grid)
    p = lio.Params.from_file(str(pf))
    obst = lio.read_obstacles(p.nx, p.ny, str(of))
    cells, av = oracle.pipe_run(p, obst)
    out = {
        "grid": grid, "nx": p.nx, "ny": p.ny, "steps": p.max_iters,
        "final_f_sha256": lattice_sha256(cells),
        "reynolds_last_av": oracle.reynolds(p, float(av[-1])),
        "total_density": float(np.sum(cells, dtype=np.float64)),
    }
    buf = _io.BytesIO()
    np.save(buf, av.astype(np.float32))
    (GOLD / "oracle_pipe" / f"{grid}.av_vels.npy.gz").write_bytes(gzip.compress(buf.getvalue(), 9))
    with tempfile.TemporaryDirectory() as wd:
        lio.write_average_velocities(os.path.join(wd, "av.dat"), av)
        fs_fix = GOLD / "check" / f"{grid}.final_state.dat.gz"
        if fs_fix.exists():
            lio.write_results(os.path.join(wd, "fs.dat"), p, obst, cells)
            res = lcheck.compare(GOLD / "check" / f"{grid}.av_vels.dat.gz", fs_fix, os.path.join(wd, "av.dat"),
                                 os.path.join(wd, "fs.dat"), 1.0)
            out["check_py"] = {"passed": res["passed"], "av_max_diff_pcnt": res["av"]["max_diff_pcnt"],
                               "fs_max_diff_pcnt": res["fs"]["max_diff_pcnt"]}
        else:
            d = lcheck.diff_values(lcheck.load_av_vels(GOLD / "check" / f"{grid}.av_vels.dat.gz"),
                                   lcheck.load_av_vels(os.path.join(wd, "av.dat")))
            out["check_py"] = {"passed": abs(d["max_diff_pcnt"]) < 1.0, "av_max_diff_pcnt": d["max_diff_pcnt"]}
    (GOLD / "oracle_pipe" / f"{grid}.json").write_text(json.dumps(out, indent=1) + "\n")
    return out


def write_final_state_fixture(grid: str, threads: int = 8) -> dict:
    """Pressure column of the oracle's final_state at full maxIters.  The
    lattice comes from the multi-threaded oracle (bitwise equal to run());
    its sha256 must equal the manifest's, so the fixture is pinned to the
    same lattice whose final_state.dat text matched the reference binary's."""
    pf, of = grid_files(grid)
    p = lio.Params.from_file(str(pf))
    obst = lio.read_obstacles(p.nx, p.ny, str(of))
    cells, _ = oracle.run_mt(p, obst, p.max_iters, threads)
    man_path = GOLD / "oracle" / f"{grid}.json"
    man = json.loads(man_path.read_text())
    if lattice_sha256(cells) != man["final_f_sha256"]:
        raise RuntimeError(f"{grid}: oracle_run_mt lattice differs from the manifest's sha256")
    _, _, _, pr = lio.macroscopic(p, obst, cells)
    pr = np.ascontiguousarray(pr, dtype=np.float32)
    buf = _io.BytesIO()
    np.save(buf, pr)
    (GOLD / "oracle" / f"{grid}.final_state_pressure.npy.gz").write_bytes(gzip.compress(buf.getvalue(), 9))
    man["final_state_pressure_sha256"] = hashlib.sha256(pr.tobytes()).hexdigest()
    man_path.write_text(json.dumps(man, indent=1) + "\n")
    return {"grid": grid, "pressure_sha256": man["final_state_pressure_sha256"]}


def small_problems():
    """Small synthetic problems for step-level bitwise vectors."""
    probs = []

    def walls(nx, ny, interior_col=None, interior_row=None):
        o = np.zeros((ny, nx), np.uint8)
        o[0, :] = 1
        o[-1, :] = 1
        o[:, 0] = 1
        o[:, -1] = 1
        if interior_col is not None:
            o[ny // 4: 3 * ny // 4, interior_col] = 1
        if interior_row is not None:
            o[interior_row, nx // 4: 3 * nx // 4] = 1
        return o

    P = lio.Params
    probs.append(("box16x8", P(16, 8, 10, 10, 0.1, 0.005, 1.85), walls(16, 8)))
    probs.append(("wall32x32", P(32, 32, 10, 10, 0.1, 0.01, 1.85), walls(32, 32, interior_col=10)))
    # periodic in y (like 128x256): side walls + a full row wall
    o = np.zeros((24, 20), np.uint8)
    o[:, 0] = 1
    o[:, -1] = 1
    o[11, :] = 1
    probs.append(("chan20x24", P(20, 24, 10, 10, 0.1, 0.005, 1.85), o))
    # ragged width (not a multiple of 4) and odd height
    probs.append(("ragged13x7", P(13, 7, 10, 10, 0.1, 0.005, 1.85), walls(13, 7, interior_row=3)))
    # fully periodic, no obstacles, random perturbation of the initial state
    probs.append(("open12x10", P(12, 10, 10, 10, 0.1, 0.005, 1.7), np.zeros((10, 12), np.uint8)))
    # a single row (ny=1: no accelerated row) and ny=2 (accelerated row is row 0)
    probs.append(("row16x1", P(16, 1, 10, 10, 0.1, 0.005, 1.85), np.zeros((1, 16), np.uint8)))
    probs.append(("two8x2", P(8, 2, 10, 10, 0.1, 0.005, 1.85), np.array([[0, 1, 0, 0, 0, 0, 0, 0]] * 2, np.uint8)))
    return probs


def make_small():
    rng = np.random.default_rng(20200625)
    arrays = {}
    meta = {}
    for name, p, obst in small_problems():
        cells0 = lio.init_cells(p)
        if name.startswith("open"):
            cells0 = (cells0 * (1 + 0.05 * rng.standard_normal(cells0.shape))).astype(np.float32)
        arrays[f"{name}/obstacles"] = obst
        arrays[f"{name}/cells0"] = cells0
        meta[name] = {"nx": p.nx, "ny": p.ny, "reynolds_dim": p.reynolds_dim, "density": p.density,
                      "accel": p.accel, "omega": p.omega}
        for n in (1, 2, 10):
            cells, av = oracle.run(p, obst, iters=n, cells=cells0)
            arrays[f"{name}/cells_after_{n}"] = cells
            arrays[f"{name}/av_{n}"] = av
    np.savez_compressed(GOLD / "small.npz", **arrays)
    (GOLD / "small.json").write_text(json.dumps(meta, indent=1) + "\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grids", default=",".join(GRIDS))
    ap.add_argument("--jobs", type=int, default=4)
    ap.add_argument("--skip-small", action="store_true")
    ap.add_argument("--pipe-grids", default="", help="also write oracle_pipe/ manifests for these grids")
    ap.add_argument("--fs-grids", default="",
                    help="only (re)write oracle/<grid>.final_state_pressure.npy.gz for these grids")
    a = ap.parse_args()
    oracle.build()
    (GOLD / "oracle").mkdir(exist_ok=True)
    if a.fs_grids:
        for g in a.fs_grids.split(","):
            print(json.dumps(write_final_state_fixture(g)))
        return
    if not a.skip_small:
        make_small()
        print("small.npz written")
    grids = [g for g in a.grids.split(",") if g]
    pipe = [g for g in a.pipe_grids.split(",") if g]
    (GOLD / "oracle_pipe").mkdir(exist_ok=True)
    with ProcessPoolExecutor(max_workers=a.jobs) as ex:
        for res in ex.map(run_grid, grids):
            print(json.dumps(res))
    for g in grids:
        print(json.dumps(write_final_state_fixture(g)))
    with ProcessPoolExecutor(max_workers=a.jobs) as ex:
        for res in ex.map(run_pipe_grid, pipe):
            print(json.dumps(res))


if __name__ == "__main__":
    main()
