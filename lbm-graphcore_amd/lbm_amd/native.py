"""ctypes binding of liblbm_hip.so (the C ABI declared in include/lbm_hip.h).

This is the Python-side mirror of the reference host's Engine usage
(main/LbmRunner.cpp:81-144): create/load/run/store/timer.  It is also the
binding a maintainer would add on the reference side.

There is deliberately no CPU fallback: if the HIP library is missing or no
GPU is visible the calls fail loudly.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

PKG_ROOT = Path(__file__).resolve().parent.parent          # lbm-graphcore_amd/
LIB_PATH = Path(os.environ.get("LBM_HIP_LIB", PKG_ROOT / "build" / "liblbm_hip.so"))

Q = 9
ABI_VERSION = 5          # LBM_ABI_VERSION in include/lbm_hip.h

LBM_OK = 0
LBM_E_INVALID, LBM_E_HIP, LBM_E_RCCL, LBM_E_NOMEM, LBM_E_STATE, LBM_E_INTERNAL = -1, -2, -3, -4, -5, -6
TRANSPORT_LOCAL, TRANSPORT_RCCL = 0, 1
KERNEL_AUTO, KERNEL_SCALAR, KERNEL_VEC4, KERNEL_STEP2, KERNEL_STREAM, KERNEL_RESIDENT, KERNEL_PIPELINE = range(7)
FLAG_FORCE_EXCHANGE, FLAG_ONE_STEP, FLAG_TOLERANCE, FLAG_PROFILE = 1, 2, 4, 8
XFER_SEND, XFER_RECV, XFER_SELF = 0, 1, 2
HALO_W1, HALO_WG = 1, 2

# every symbol include/lbm_hip.h declares
EXPORTED = [
    "lbm_abi_version", "lbm_partition", "lbm_halo_plan", "lbm_exchange_schedule", "lbm_device_count",
    "lbm_rccl_unique_id",
    "lbm_create", "lbm_create_ex", "lbm_load_cells", "lbm_init_equilibrium",
    "lbm_run", "lbm_run_steps", "lbm_store", "lbm_load_cells_local", "lbm_store_local", "lbm_local_cells",
    "lbm_last_run_seconds",
    "lbm_total_free_cells", "lbm_local_rects", "lbm_kernel_in_use", "lbm_steps_per_launch",
    "lbm_run_stats", "lbm_profile_summary", "lbm_profile_reset", "lbm_placement_probe", "lbm_numerics", "lbm_nonfinite_count", "lbm_source_hash",
    "lbm_last_error", "lbm_destroy",
]
# every symbol include/lbm3d_hip.h declares (D3Q19 extension)
EXPORTED3D = [
    "lbm3d_create", "lbm3d_init_equilibrium", "lbm3d_load_cells", "lbm3d_run_steps", "lbm3d_store",
    "lbm3d_last_run_seconds", "lbm3d_total_free_cells", "lbm3d_local_slabs", "lbm3d_exchange_schedule",
    "lbm3d_last_error", "lbm3d_destroy",
]
Q3 = 19


class LbmError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"lbm error {code}: {msg}")
        self.code = code


class Params(ctypes.Structure):
    """lbm_params (mirror of lbm::Params, main/include/LbmParams.hpp:16-65)."""
    _fields_ = [
        ("nx", ctypes.c_int32),
        ("ny", ctypes.c_int32),
        ("max_iters", ctypes.c_int32),
        ("reynolds_dim", ctypes.c_int32),
        ("density", ctypes.c_float),
        ("accel", ctypes.c_float),
        ("omega", ctypes.c_float),
    ]


class Config(ctypes.Structure):
    _fields_ = [
        ("parts", ctypes.c_int32),
        ("grid_rows", ctypes.c_int32),
        ("grid_cols", ctypes.c_int32),
        ("transport", ctypes.c_int32),
        ("rank", ctypes.c_int32),
        ("world", ctypes.c_int32),
        ("devices", ctypes.POINTER(ctypes.c_int32)),
        ("num_devices", ctypes.c_int32),
        ("rccl_unique_id", ctypes.POINTER(ctypes.c_uint8)),
        ("kernel", ctypes.c_int32),
        ("graph_steps", ctypes.c_int32),
        ("flags", ctypes.c_int32),
        ("steps_per_launch", ctypes.c_int32),
    ]


class Params3D(ctypes.Structure):
    """lbm3d_params (include/lbm3d_hip.h)."""
    _fields_ = [("nx", ctypes.c_int32), ("ny", ctypes.c_int32), ("nz", ctypes.c_int32), ("max_iters", ctypes.c_int32),
                ("density", ctypes.c_float), ("accel", ctypes.c_float), ("omega", ctypes.c_float)]


class Rect(ctypes.Structure):
    _fields_ = [("x0", ctypes.c_int32), ("y0", ctypes.c_int32), ("w", ctypes.c_int32), ("h", ctypes.c_int32)]


class KernelTime(ctypes.Structure):
    """lbm_kernel_time (include/lbm_hip.h)."""
    _fields_ = [("name", ctypes.c_char * 64), ("launches", ctypes.c_int64), ("total_ms", ctypes.c_double),
                ("min_ms", ctypes.c_double), ("max_ms", ctypes.c_double)]


class Xfer(ctypes.Structure):
    """lbm_xfer (include/lbm_hip.h): one post of a halo exchange."""
    _fields_ = [("op", ctypes.c_int32), ("dir", ctypes.c_int32), ("peer", ctypes.c_int32),
                ("reserved", ctypes.c_int32), ("floats", ctypes.c_int64)]


_lib = None


def load_library() -> ctypes.CDLL:
    """Load liblbm_hip.so and declare every C-ABI signature (no GPU needed).

    Refuses a library whose compiled-in source hash (lbm_source_hash) differs
    from the hash of the csrc/ and include/ sources beside it: a stale build
    fails loudly instead of silently running old kernels."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise FileNotFoundError(
            f"{LIB_PATH} not found: build the HIP library first (make -C lbm-graphcore_amd "
            "or __graft_entry__.build()); there is no CPU fallback")
    L = ctypes.CDLL(str(LIB_PATH))
    L.lbm_source_hash.argtypes = []
    L.lbm_source_hash.restype = ctypes.c_char_p
    built = L.lbm_source_hash().decode()
    from . import srchash
    if srchash.source_files() and built != srchash.source_hash():
        raise RuntimeError(f"{LIB_PATH} was built from other sources (hash {built}, sources "
                           f"{srchash.source_hash()}): rebuild it (make -C lbm-graphcore_amd)")
    H = ctypes.c_void_p
    i32, i64 = ctypes.c_int32, ctypes.c_int64
    f32p = ctypes.POINTER(ctypes.c_float)
    u8p = ctypes.POINTER(ctypes.c_uint8)
    i32p = ctypes.POINTER(ctypes.c_int32)
    sig = {
        "lbm_abi_version": ([], i32),
        "lbm_partition": ([i32, i32, i32, i32, i32, i32p, i32p, ctypes.POINTER(Rect)], ctypes.c_int),
        "lbm_halo_plan": ([i32p], ctypes.c_int),
        "lbm_exchange_schedule": ([i32, i32, i32, i32, i32, i32, i32, i32, i32, ctypes.POINTER(Xfer), i32, i32p],
                                  ctypes.c_int),
        "lbm3d_exchange_schedule": ([i32, i32, i32, i32, i32, i32, ctypes.POINTER(Xfer), i32, i32p], ctypes.c_int),
        "lbm_device_count": ([], i32),
        "lbm_rccl_unique_id": ([u8p], ctypes.c_int),
        "lbm_create": ([ctypes.POINTER(Params), u8p, i32, ctypes.POINTER(H)], ctypes.c_int),
        "lbm_create_ex": ([ctypes.POINTER(Params), u8p, ctypes.POINTER(Config), ctypes.POINTER(H)], ctypes.c_int),
        "lbm_load_cells": ([H, f32p], ctypes.c_int),
        "lbm_init_equilibrium": ([H], ctypes.c_int),
        "lbm_run": ([H], ctypes.c_int),
        "lbm_run_steps": ([H, i32, i32], ctypes.c_int),
        "lbm_store": ([H, f32p, f32p, i32], ctypes.c_int),
        "lbm_load_cells_local": ([H, f32p], ctypes.c_int),
        "lbm_store_local": ([H, f32p, f32p, i32], ctypes.c_int),
        "lbm_local_cells": ([H], i64),
        "lbm_last_run_seconds": ([H, ctypes.POINTER(ctypes.c_double)], ctypes.c_int),
        "lbm_total_free_cells": ([H], i64),
        "lbm_local_rects": ([H, ctypes.POINTER(Rect), i32, i32p], ctypes.c_int),
        "lbm_kernel_in_use": ([H], i32),
        "lbm_steps_per_launch": ([H], i32),
        "lbm_run_stats": ([H, i32p, i32p], ctypes.c_int),
        "lbm_profile_summary": ([H, ctypes.POINTER(KernelTime), i32, i32p], ctypes.c_int),
        "lbm_profile_reset": ([H], ctypes.c_int),
        "lbm_placement_probe": ([H, i32p, i32p, f32p, i32], ctypes.c_int),
        "lbm_numerics": ([H], i32),
        "lbm_nonfinite_count": ([H, ctypes.POINTER(i64)], ctypes.c_int),
        "lbm_last_error": ([H], ctypes.c_char_p),
        "lbm_destroy": ([H], None),
        "lbm3d_create": ([ctypes.POINTER(Params3D), u8p, ctypes.POINTER(Config), ctypes.POINTER(H)], ctypes.c_int),
        "lbm3d_init_equilibrium": ([H], ctypes.c_int),
        "lbm3d_load_cells": ([H, f32p], ctypes.c_int),
        "lbm3d_run_steps": ([H, i32], ctypes.c_int),
        "lbm3d_store": ([H, f32p, f32p, i32], ctypes.c_int),
        "lbm3d_last_run_seconds": ([H, ctypes.POINTER(ctypes.c_double)], ctypes.c_int),
        "lbm3d_total_free_cells": ([H], i64),
        "lbm3d_local_slabs": ([H, i32p, i32p, i32, i32p], ctypes.c_int),
        "lbm3d_last_error": ([H], ctypes.c_char_p),
        "lbm3d_destroy": ([H], None),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    if L.lbm_abi_version() != ABI_VERSION:
        raise RuntimeError(f"{LIB_PATH}: ABI version {L.lbm_abi_version()}, binding expects {ABI_VERSION}")
    _lib = L
    return L


def _f32(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def partition(nx: int, ny: int, parts: int, grid_rows: int = 0, grid_cols: int = 0):
    """Reference partition rule via the C ABI. Returns (rows, cols, [(x0,y0,w,h)...])."""
    L = load_library()
    rects = (Rect * parts)()
    r, c = ctypes.c_int32(), ctypes.c_int32()
    rc = L.lbm_partition(nx, ny, parts, grid_rows, grid_cols, ctypes.byref(r), ctypes.byref(c), rects)
    if rc != LBM_OK:
        raise LbmError(rc, f"cannot partition {nx}x{ny} into {parts}")
    return r.value, c.value, [(q.x0, q.y0, q.w, q.h) for q in rects]


def halo_plan():
    """[(dx, dy, [planes...]) for the 8 directions E, N, W, S, NE, NW, SW, SE]."""
    t = (ctypes.c_int32 * 48)()
    rc = load_library().lbm_halo_plan(t)
    if rc != LBM_OK:
        raise LbmError(rc, "lbm_halo_plan failed")
    out = []
    for d in range(8):
        dx, dy, n = t[6 * d], t[6 * d + 1], t[6 * d + 2]
        out.append((dx, dy, [t[6 * d + 3 + i] for i in range(n)]))
    return out


def exchange_schedule(nx: int, ny: int, parts: int, rank: int, mode: int = HALO_WG, halo_width: int = 1,
                      grid_rows: int = 0, grid_cols: int = 0, force_exchange: bool = False):
    """The engine's own ordered halo-exchange posts for `rank` (lbm_exchange_schedule):
    [(op, dir, peer, floats), ...] with op XFER_SEND / XFER_RECV / XFER_SELF."""
    L = load_library()
    buf = (Xfer * 32)()
    n = ctypes.c_int32()
    rc = L.lbm_exchange_schedule(nx, ny, parts, grid_rows, grid_cols, rank, mode, halo_width, int(force_exchange),
                                 buf, 32, ctypes.byref(n))
    if rc != LBM_OK:
        raise LbmError(rc, f"lbm_exchange_schedule({nx}, {ny}, {parts}, rank {rank}) failed")
    return [(x.op, x.dir, x.peer, x.floats) for x in buf[:n.value]]


def exchange_schedule3d(nx: int, ny: int, nz: int, parts: int, rank: int, planes: int):
    """The D3Q19 engine's ordered z-slab exchange posts (lbm3d_exchange_schedule);
    dir 0 = +z (up), 1 = -z (down)."""
    L = load_library()
    buf = (Xfer * 4)()
    n = ctypes.c_int32()
    rc = L.lbm3d_exchange_schedule(nx, ny, nz, parts, rank, planes, buf, 4, ctypes.byref(n))
    if rc != LBM_OK:
        raise LbmError(rc, f"lbm3d_exchange_schedule({nx}, {ny}, {nz}, {parts}, rank {rank}) failed")
    return [(x.op, x.dir, x.peer, x.floats) for x in buf[:n.value]]


def device_count() -> int:
    return int(load_library().lbm_device_count())


def rccl_unique_id() -> bytes:
    buf = (ctypes.c_uint8 * 128)()
    rc = load_library().lbm_rccl_unique_id(buf)
    if rc != LBM_OK:
        raise LbmError(rc, "ncclGetUniqueId failed")
    return bytes(buf)


class Engine:
    """One lbm_handle: the HIP counterpart of the reference's poplar::Engine."""

    def __init__(self, params, obstacles: np.ndarray, num_gpus: int = 1, *, parts: int | None = None,
                 grid=(0, 0), transport: int = TRANSPORT_LOCAL, rank: int = 0, world: int = 1,
                 devices=None, unique_id: bytes | None = None, kernel: int = KERNEL_AUTO,
                 graph_steps: int = 0, flags: int = 0, steps_per_launch: int = 0):
        self._L = load_library()
        self.params = Params(int(params.nx), int(params.ny), int(params.max_iters), int(params.reynolds_dim),
                             float(params.density), float(params.accel), float(params.omega))
        obst = np.ascontiguousarray(obstacles, dtype=np.uint8)
        if obst.size != self.params.nx * self.params.ny:
            raise ValueError("obstacles must have ny*nx entries")
        self._h = ctypes.c_void_p()
        cfg = Config()
        cfg.parts = int(parts if parts is not None else (world if transport == TRANSPORT_RCCL else num_gpus))
        cfg.grid_rows, cfg.grid_cols = int(grid[0]), int(grid[1])
        cfg.transport = transport
        cfg.rank, cfg.world = int(rank), int(world)
        if devices:
            self._devs = (ctypes.c_int32 * len(devices))(*devices)
            cfg.devices = self._devs
            cfg.num_devices = len(devices)
        if unique_id is not None:
            self._uid = (ctypes.c_uint8 * 128).from_buffer_copy(unique_id)
            cfg.rccl_unique_id = self._uid
        cfg.kernel = kernel
        cfg.graph_steps = graph_steps
        cfg.flags = flags
        cfg.steps_per_launch = int(steps_per_launch)
        rc = self._L.lbm_create_ex(ctypes.byref(self.params), obst.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                   ctypes.byref(cfg), ctypes.byref(self._h))
        if rc != LBM_OK:
            raise LbmError(rc, self._L.lbm_last_error(None).decode())

    def _check(self, rc: int):
        if rc != LBM_OK:
            raise LbmError(rc, self._L.lbm_last_error(self._h).decode())

    def load_cells(self, cells: np.ndarray) -> None:
        c = np.ascontiguousarray(cells, dtype=np.float32)
        if c.size != self.params.nx * self.params.ny * Q:
            raise ValueError("cells must be AoS float32[ny][nx][9]")
        self._check(self._L.lbm_load_cells(self._h, _f32(c)))

    def init_equilibrium(self) -> None:
        self._check(self._L.lbm_init_equilibrium(self._h))

    def run(self) -> None:
        self._check(self._L.lbm_run(self._h))

    def run_steps(self, steps: int, accelerate_first: bool = False) -> None:
        self._check(self._L.lbm_run_steps(self._h, int(steps), 1 if accelerate_first else 0))

    def store(self, cells: bool = True, n_av: int | None = None):
        """Returns (cells AoS float32[ny][nx][9] or None, av_vels float32[n_av])."""
        n_av = int(self.params.max_iters if n_av is None else n_av)
        out = np.zeros((self.params.ny, self.params.nx, Q), np.float32) if cells else None
        av = np.zeros(max(n_av, 1), np.float32)
        self._check(self._L.lbm_store(self._h, _f32(out) if cells else None, _f32(av), n_av))
        return out, av[:n_av]

    def load_cells_local(self, blocks) -> None:
        """This handle's sub-domains only: one AoS float32[h][w][9] per local rect
        (local_rects() order), as lbm_load_cells_local takes them packed."""
        rects = self.local_rects()
        if len(blocks) != len(rects):
            raise ValueError("one block per local rect")
        for b, (_, _, w, h) in zip(blocks, rects):
            if tuple(np.shape(b)) != (h, w, Q):
                raise ValueError(f"block shape {np.shape(b)} != {(h, w, Q)}")
        packed = np.ascontiguousarray(np.concatenate([np.asarray(b, np.float32).reshape(-1) for b in blocks]))
        assert packed.size == int(self._L.lbm_local_cells(self._h)) * Q
        self._check(self._L.lbm_load_cells_local(self._h, _f32(packed)))

    def store_local(self, cells: bool = True, n_av: int | None = None):
        """Returns ([AoS float32[h][w][9] per local rect] or None, av_vels float32[n_av])."""
        n_av = int(self.params.max_iters if n_av is None else n_av)
        rects = self.local_rects()
        packed = np.zeros(int(self._L.lbm_local_cells(self._h)) * Q, np.float32) if cells else None
        av = np.zeros(max(n_av, 1), np.float32)
        self._check(self._L.lbm_store_local(self._h, _f32(packed) if cells else None, _f32(av), n_av))
        if not cells:
            return None, av[:n_av]
        out, off = [], 0
        for (_, _, w, h) in rects:
            out.append(packed[off:off + w * h * Q].reshape(h, w, Q))
            off += w * h * Q
        return out, av[:n_av]

    def last_run_seconds(self) -> float:
        s = ctypes.c_double()
        self._check(self._L.lbm_last_run_seconds(self._h, ctypes.byref(s)))
        return s.value

    def total_free_cells(self) -> int:
        return int(self._L.lbm_total_free_cells(self._h))

    def local_rects(self):
        n = ctypes.c_int32()
        self._check(self._L.lbm_local_rects(self._h, None, 0, ctypes.byref(n)))
        rects = (Rect * max(n.value, 1))()
        self._check(self._L.lbm_local_rects(self._h, rects, n.value, ctypes.byref(n)))
        return [(q.x0, q.y0, q.w, q.h) for q in rects[:n.value]]

    def kernel_in_use(self) -> str:
        return {KERNEL_SCALAR: "scalar", KERNEL_VEC4: "vec4", KERNEL_STEP2: "step2", KERNEL_STREAM: "stream",
                KERNEL_RESIDENT: "resident", KERNEL_PIPELINE: "pipeline"}[
            int(self._L.lbm_kernel_in_use(self._h))]

    def steps_per_launch(self) -> int:
        return int(self._L.lbm_steps_per_launch(self._h))

    def run_stats(self):
        """(fused launches, one-step launches) of the last run."""
        a, b = ctypes.c_int32(), ctypes.c_int32()
        self._check(self._L.lbm_run_stats(self._h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def profile_summary(self):
        """[{name, launches, total_ms, min_ms, max_ms}] per launch class (LBM_FLAG_PROFILE handles)."""
        n = ctypes.c_int32()
        self._check(self._L.lbm_profile_summary(self._h, None, 0, ctypes.byref(n)))
        buf = (KernelTime * max(n.value, 1))()
        self._check(self._L.lbm_profile_summary(self._h, buf, n.value, ctypes.byref(n)))
        return [{"name": k.name.decode(), "launches": k.launches, "total_ms": k.total_ms, "min_ms": k.min_ms,
                 "max_ms": k.max_ms} for k in buf[:n.value]]

    def profile_reset(self) -> None:
        self._check(self._L.lbm_profile_reset(self._h))

    def placement(self):
        """(kept pair or -1, [ms per launch of each pair tried]) of the placement probe."""
        kept, tried = ctypes.c_int32(), ctypes.c_int32()
        ms = (ctypes.c_float * 16)()
        self._check(self._L.lbm_placement_probe(self._h, ctypes.byref(kept), ctypes.byref(tried), ms, 16))
        return kept.value, [ms[i] for i in range(min(tried.value, 16))]

    def nonfinite_count(self) -> int:
        """NaN / Inf populations in the current lattice (device scan)."""
        n = ctypes.c_int64()
        self._check(self._L.lbm_nonfinite_count(self._h, ctypes.byref(n)))
        return n.value

    def numerics(self) -> str:
        """'bitwise' (every kernel equals the CPU oracle) or 'tolerance' (LBM_FLAG_TOLERANCE collision)."""
        return "tolerance" if int(self._L.lbm_numerics(self._h)) == 1 else "bitwise"

    def close(self) -> None:
        if self._h:
            self._L.lbm_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Engine3D:
    """One lbm3d_handle: the D3Q19 extension engine (include/lbm3d_hip.h)."""

    def __init__(self, params, obstacles: np.ndarray, *, parts: int = 1, transport: int = TRANSPORT_LOCAL,
                 rank: int = 0, world: int = 1, devices=None, unique_id: bytes | None = None, flags: int = 0):
        self._L = load_library()
        self.params = Params3D(int(params.nx), int(params.ny), int(params.nz), int(params.max_iters),
                               float(params.density), float(params.accel), float(params.omega))
        obst = np.ascontiguousarray(obstacles, dtype=np.uint8)
        if obst.size != self.params.nx * self.params.ny * self.params.nz:
            raise ValueError("obstacles must have nz*ny*nx entries")
        cfg = Config()
        cfg.parts = int(world if transport == TRANSPORT_RCCL else parts)
        cfg.transport = transport
        cfg.flags = int(flags)  # FLAG_TOLERANCE: the two-step passes use the reciprocal collision
        cfg.rank, cfg.world = int(rank), int(world)
        if devices:
            self._devs = (ctypes.c_int32 * len(devices))(*devices)
            cfg.devices = self._devs
            cfg.num_devices = len(devices)
        if unique_id is not None:
            self._uid = (ctypes.c_uint8 * 128).from_buffer_copy(unique_id)
            cfg.rccl_unique_id = self._uid
        self._h = ctypes.c_void_p()
        rc = self._L.lbm3d_create(ctypes.byref(self.params), obst.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                  ctypes.byref(cfg), ctypes.byref(self._h))
        if rc != LBM_OK:
            raise LbmError(rc, self._L.lbm3d_last_error(None).decode())

    def _check(self, rc: int):
        if rc != LBM_OK:
            raise LbmError(rc, self._L.lbm3d_last_error(self._h).decode())

    def init_equilibrium(self) -> None:
        self._check(self._L.lbm3d_init_equilibrium(self._h))

    def load_cells(self, cells: np.ndarray) -> None:
        c = np.ascontiguousarray(cells, dtype=np.float32)
        if c.size != self.params.nx * self.params.ny * self.params.nz * Q3:
            raise ValueError("cells must be AoS float32[nz][ny][nx][19]")
        self._check(self._L.lbm3d_load_cells(self._h, _f32(c)))

    def run_steps(self, steps: int) -> None:
        self._check(self._L.lbm3d_run_steps(self._h, int(steps)))

    def store(self, cells: bool = True, n_av: int = 0):
        out = np.zeros((self.params.nz, self.params.ny, self.params.nx, Q3), np.float32) if cells else None
        av = np.zeros(max(int(n_av), 1), np.float32)
        self._check(self._L.lbm3d_store(self._h, _f32(out) if cells else None, _f32(av), int(n_av)))
        return out, av[:int(n_av)]

    def last_run_seconds(self) -> float:
        s = ctypes.c_double()
        self._check(self._L.lbm3d_last_run_seconds(self._h, ctypes.byref(s)))
        return s.value

    def total_free_cells(self) -> int:
        return int(self._L.lbm3d_total_free_cells(self._h))

    def local_slabs(self):
        n = ctypes.c_int32()
        z0 = (ctypes.c_int32 * 64)()
        nz = (ctypes.c_int32 * 64)()
        self._check(self._L.lbm3d_local_slabs(self._h, z0, nz, 64, ctypes.byref(n)))
        return [(z0[i], nz[i]) for i in range(n.value)]

    def close(self) -> None:
        if self._h:
            self._L.lbm3d_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
