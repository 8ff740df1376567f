"""TEST INFRASTRUCTURE ONLY -- ctypes front end of the CPU oracle.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg
import this module, and only as the checker / reported CPU baseline.  The
product (``lbm-graphcore_amd/``) never imports it.

Wraps ``oracle/liblbm_oracle.so`` (built from ``oracle/lbm_oracle.c``, a
restatement of ``main/LastChance.cpp:156-267`` of the reference) and, for
the reference-run helpers, ``oracle/_ref/lastchance`` (the reference's own
CPU program compiled from its sources by ``oracle/Makefile``).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import tempfile
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "liblbm_oracle.so"
REF_LASTCHANCE = HERE / "_ref" / "lastchance"
REF_LBMCPU = HERE / "_ref" / "lbm_cpu"

Q = 9


class OracleParams(ctypes.Structure):
    _fields_ = [
        ("nx", ctypes.c_int32),
        ("ny", ctypes.c_int32),
        ("max_iters", ctypes.c_int32),
        ("reynolds_dim", ctypes.c_int32),
        ("density", ctypes.c_float),
        ("accel", ctypes.c_float),
        ("omega", ctypes.c_float),
    ]


_lib = None


def build() -> None:
    """Compile the restatement (and the reference binaries when sources exist)."""
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = ctypes.CDLL(str(LIB_PATH))
        P = ctypes.POINTER(OracleParams)
        f32p = ctypes.POINTER(ctypes.c_float)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.oracle_init_equilibrium.argtypes = [P, f32p]
        L.oracle_free_cells.argtypes = [P, u8p]
        L.oracle_free_cells.restype = ctypes.c_int64
        L.oracle_accelerate.argtypes = [P, f32p, u8p]
        L.oracle_step.argtypes = [P, f32p, f32p, u8p]
        L.oracle_step.restype = ctypes.c_float
        L.oracle_step_ghosted.argtypes = [P, ctypes.c_int, ctypes.c_int, f32p, f32p, u8p, ctypes.c_int]
        L.oracle_step_ghosted.restype = ctypes.c_float
        L.oracle_run.argtypes = [P, f32p, u8p, ctypes.c_int, f32p]
        L.oracle_run.restype = ctypes.c_int
        L.oracle_av_velocity.argtypes = [P, f32p, u8p]
        L.oracle_av_velocity.restype = ctypes.c_float
        L.oracle_run_mt.argtypes = [P, f32p, u8p, ctypes.c_int, f32p, ctypes.c_int]
        L.oracle_run_mt.restype = ctypes.c_int
        L.oracle_pipe_run.argtypes = [P, f32p, u8p, ctypes.c_int, f32p]
        L.oracle_pipe_run.restype = ctypes.c_int
        P3 = ctypes.POINTER(Oracle3DParams)
        L.oracle3d_init_equilibrium.argtypes = [P3, f32p]
        L.oracle3d_free_cells.argtypes = [P3, u8p]
        L.oracle3d_free_cells.restype = ctypes.c_int64
        L.oracle3d_step.argtypes = [P3, f32p, f32p, u8p]
        L.oracle3d_step.restype = ctypes.c_float
        L.oracle3d_run.argtypes = [P3, f32p, u8p, ctypes.c_int, f32p]
        L.oracle3d_step_slab.argtypes = [P3, ctypes.c_int, f32p, f32p, u8p]
        L.oracle3d_step_slab.restype = ctypes.c_float
        L.oracle3d_run.restype = ctypes.c_int
        L.oracle_reynolds.argtypes = [P, ctypes.c_float]
        L.oracle_reynolds.restype = ctypes.c_float
        _lib = L
    return _lib


class Oracle3DParams(ctypes.Structure):
    _fields_ = [("nx", ctypes.c_int32), ("ny", ctypes.c_int32), ("nz", ctypes.c_int32), ("max_iters", ctypes.c_int32),
                ("density", ctypes.c_float), ("accel", ctypes.c_float), ("omega", ctypes.c_float)]


def _p3(p) -> Oracle3DParams:
    return Oracle3DParams(int(p.nx), int(p.ny), int(p.nz), int(p.max_iters), float(p.density), float(p.accel),
                          float(p.omega))


def init_cells3d(params) -> np.ndarray:
    """D3Q19 equilibrium at rest, AoS float32[nz][ny][nx][19] (oracle/lbm_oracle3d.c)."""
    cells = np.empty((params.nz, params.ny, params.nx, 19), np.float32)
    lib().oracle3d_init_equilibrium(ctypes.byref(_p3(params)), _f(cells))
    return cells


def free_cells3d(params, obst: np.ndarray) -> int:
    return int(lib().oracle3d_free_cells(ctypes.byref(_p3(params)), _u8(np.ascontiguousarray(obst, np.uint8))))


def run3d(params, obst: np.ndarray, iters: int, cells: np.ndarray | None = None):
    """D3Q19 restatement: `iters` steps. Returns (final_cells, av_vels[iters]). Parity unpinned
    w.r.t. the reference (no 3-D code upstream)."""
    if cells is None:
        cells = init_cells3d(params)
    cells = np.ascontiguousarray(cells, dtype=np.float32).copy()
    av = np.zeros(max(int(iters), 1), np.float32)
    rc = lib().oracle3d_run(ctypes.byref(_p3(params)), _f(cells), _u8(np.ascontiguousarray(obst, np.uint8)),
                            int(iters), _f(av))
    if rc != 0:
        raise MemoryError("oracle3d_run allocation failed")
    return cells, av[:int(iters)]


def step3d_slab(params, ghosted: np.ndarray, obst_slab: np.ndarray):
    """One D3Q19 step of a z slab given its ghosted input [(nzs+2)][ny][nx][19].
    Returns (out [nzs][ny][nx][19], tot_u)."""
    nzs = ghosted.shape[0] - 2
    out = np.empty((nzs, params.ny, params.nx, 19), np.float32)
    tot = lib().oracle3d_step_slab(ctypes.byref(_p3(params)), nzs, _f(np.ascontiguousarray(ghosted, np.float32)),
                                   _f(out), _u8(np.ascontiguousarray(obst_slab, np.uint8)))
    return out, float(np.float32(tot))


def _p(params) -> OracleParams:
    return OracleParams(int(params.nx), int(params.ny), int(params.max_iters),
                        int(params.reynolds_dim), float(params.density),
                        float(params.accel), float(params.omega))


def _f(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _u8(a: np.ndarray):
    assert a.dtype == np.uint8 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def init_cells(params) -> np.ndarray:
    cells = np.empty((params.ny, params.nx, Q), np.float32)
    lib().oracle_init_equilibrium(ctypes.byref(_p(params)), _f(cells))
    return cells


def free_cells(params, obst: np.ndarray) -> int:
    return int(lib().oracle_free_cells(ctypes.byref(_p(params)), _u8(obst)))


def accelerate(params, cells: np.ndarray, obst: np.ndarray) -> None:
    lib().oracle_accelerate(ctypes.byref(_p(params)), _f(cells), _u8(obst))


def step(params, cells: np.ndarray, obst: np.ndarray):
    """One fused periodic step. Returns (new_cells, tot_u)."""
    out = np.empty_like(cells)
    tot = lib().oracle_step(ctypes.byref(_p(params)), _f(cells), _f(out), _u8(obst))
    return out, float(np.float32(tot))


def step_ghosted(params, ghosted: np.ndarray, obst: np.ndarray, accel_row: int):
    """Step a sub-block given its (h+2, w+2, 9) ghosted input. Returns (out, tot_u)."""
    h, w = ghosted.shape[0] - 2, ghosted.shape[1] - 2
    out = np.empty((h, w, Q), np.float32)
    ob = np.ascontiguousarray(obst, dtype=np.uint8)
    tot = lib().oracle_step_ghosted(ctypes.byref(_p(params)), w, h,
                                    _f(np.ascontiguousarray(ghosted)), _f(out), _u8(ob), accel_row)
    return out, float(np.float32(tot))


def run(params, obst: np.ndarray, iters: int | None = None, cells: np.ndarray | None = None,
        accelerate_first: bool = True):
    """Accelerate once (unless accelerate_first=False: a continuation run, as
    lbm_run_steps(..., 0)), then `iters` steps. Returns (final_cells, av_vels[iters])."""
    iters = int(params.max_iters if iters is None else iters)
    if cells is None:
        cells = init_cells(params)
    if not accelerate_first:
        ob = np.ascontiguousarray(obst, np.uint8)
        fc = np.float32(free_cells(params, ob))
        cur = np.ascontiguousarray(cells, dtype=np.float32).copy()
        av = np.zeros(iters, np.float32)
        for t in range(iters):
            cur, tot = step(params, cur, ob)
            av[t] = np.float32(tot) / fc
        return cur, av
    cells = np.ascontiguousarray(cells, dtype=np.float32).copy()
    av = np.zeros(max(iters, 1), np.float32)
    rc = lib().oracle_run(ctypes.byref(_p(params)), _f(cells), _u8(np.ascontiguousarray(obst, np.uint8)),
                          iters, _f(av))
    if rc != 0:
        raise MemoryError("oracle_run allocation failed")
    return cells, av[:iters]


def run_mt(params, obst: np.ndarray, iters: int, threads: int, cells: np.ndarray | None = None):
    """oracle_run on `threads` OpenMP threads (informational all-cores CPU baseline);
    the lattice is bitwise equal to run()."""
    if cells is None:
        cells = init_cells(params)
    cells = np.ascontiguousarray(cells, dtype=np.float32).copy()
    av = np.zeros(max(int(iters), 1), np.float32)
    rc = lib().oracle_run_mt(ctypes.byref(_p(params)), _f(cells), _u8(np.ascontiguousarray(obst, np.uint8)),
                             int(iters), _f(av), int(threads))
    if rc != 0:
        raise MemoryError("oracle_run_mt allocation failed")
    return cells, av[:int(iters)]


def pipe_run(params, obst: np.ndarray, iters: int | None = None, cells: np.ndarray | None = None):
    """Unfused pipeline (accelerate -> propagate -> rebound -> textbook collision ->
    av_velocity) `iters` times. Returns (final_cells, av_vels[iters])."""
    iters = int(params.max_iters if iters is None else iters)
    if cells is None:
        cells = init_cells(params)
    cells = np.ascontiguousarray(cells, dtype=np.float32).copy()
    av = np.zeros(max(iters, 1), np.float32)
    rc = lib().oracle_pipe_run(ctypes.byref(_p(params)), _f(cells), _u8(np.ascontiguousarray(obst, np.uint8)),
                               iters, _f(av))
    if rc != 0:
        raise MemoryError("oracle_pipe_run allocation failed")
    return cells, av[:iters]


def av_velocity(params, cells: np.ndarray, obst: np.ndarray) -> float:
    return float(lib().oracle_av_velocity(ctypes.byref(_p(params)), _f(cells), _u8(obst)))


def reynolds(params, av: float) -> float:
    return float(lib().oracle_reynolds(ctypes.byref(_p(params)), ctypes.c_float(av)))


def run_reference(params_file: str, obstacles_file: str, workdir: str | None = None,
                  binary: Path = REF_LASTCHANCE) -> dict:
    """Run the reference's own LastChance binary; return its outputs and timing."""
    if not binary.exists():
        raise FileNotFoundError(f"{binary} not built (needs /root/reference at build time)")
    wd = workdir or tempfile.mkdtemp(prefix="lbm_ref_")
    proc = subprocess.run([str(binary), os.path.abspath(params_file), os.path.abspath(obstacles_file)],
                          cwd=wd, capture_output=True, text=True, check=True)
    out = {"stdout": proc.stdout, "workdir": wd,
           "av_vels": os.path.join(wd, "av_vels.dat"),
           "final_state": os.path.join(wd, "final_state.dat")}
    for line in proc.stdout.splitlines():
        if line.startswith("Elapsed time:"):
            out["elapsed_s"] = float(line.split()[2])
        if line.startswith("Reynolds number:"):
            out["reynolds"] = float(line.split()[2])
    return out


def run_lbm_cpu(params_file: str, obstacles_file: str, workdir: str | None = None,
                binary: Path = REF_LBMCPU) -> dict:
    """Run the reference's main/LbmCpu.cpp as committed (oracle/_ref/lbm_cpu) --
    a cost-only baseline: its live kernel is numerically broken upstream
    (SURVEY.md 8c), so its outputs are not checked.  Its timed region
    (LbmCpu.cpp:404-419) includes a full-lattice printf, sent to a file here.
    Returns {"compute_s": the program's own "Total compute time", ...}."""
    if not binary.exists():
        raise FileNotFoundError(f"{binary} not built (needs /root/reference at build time)")
    wd = workdir or tempfile.mkdtemp(prefix="lbm_cpu_")
    with open(os.path.join(wd, "stdout.txt"), "w") as so:
        proc = subprocess.run([str(binary), "--params", os.path.abspath(params_file),
                               "--obstacles", os.path.abspath(obstacles_file)],
                              cwd=wd, stdout=so, stderr=subprocess.PIPE, text=True, check=True)
    out = {"workdir": wd, "stderr": proc.stderr}
    with open(os.path.join(wd, "stdout.txt")) as f:
        for line in f:
            if line.startswith("Total compute time was"):
                out["compute_s"] = float(line.split()[-1].rstrip("s"))
    return out


def cpu_model() -> str:
    """Host CPU model name (/proc/cpuinfo) and logical CPU count."""
    name = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    name = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return f"{name} ({os.cpu_count()} logical CPUs visible)"
