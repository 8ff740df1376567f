"""Problem I/O, mirroring the reference host (kept on the host in this build).

* Params.from_file      -- lbm::Params::fromFile     main/include/LbmParams.hpp:28-58
* Obstacles.from_file   -- lbm::Obstacles::fromFile  main/include/LbmParams.hpp:92-123
* init_cells            -- lbm::Cells::initialise    main/include/LatticeBoltzmannUtils.hpp:137-157
* write_average_velocities -- writeAverageVelocities  LatticeBoltzmannUtils.hpp:208-219
* write_results         -- writeResults              LatticeBoltzmannUtils.hpp:221-281
* reynolds_number       -- reynoldsNumber            LatticeBoltzmannUtils.hpp:202-205

Error behaviour follows the reference: loaders return None (std::nullopt)
and print the reference's message on stderr.  One deliberate strengthening:
an obstacle outside the grid is rejected (the reference indexes out of
bounds; LastChance.cpp:476-478 rejects it too).
"""
from __future__ import annotations

import sys
from dataclasses import dataclass

import numpy as np

Q = 9
C_SQ = np.float32(1.0) / np.float32(3.0)


@dataclass(frozen=True)
class Params:
    nx: int
    ny: int
    max_iters: int
    reynolds_dim: int
    density: float   # fp32 values (stof)
    accel: float
    omega: float

    @staticmethod
    def from_file(filename: str) -> "Params | None":
        """7 lines: nx, ny, maxIters, reynolds_dim (stoul), density, accel, omega (stof)."""
        try:
            with open(filename, "r") as f:
                lines = f.read().split("\n")
        except OSError:
            print(f"Could not read parameters from {filename}", file=sys.stderr)
            return None
        try:
            ints = [int(lines[i].strip().split()[0]) for i in range(4)]
            floats = [float(np.float32(lines[i].strip().split()[0])) for i in range(4, 7)]
        except (IndexError, ValueError):
            print(f"Could not read parameters from {filename}", file=sys.stderr)
            return None
        if any(v < 0 for v in ints):
            print(f"Could not read parameters from {filename}", file=sys.stderr)
            return None
        return Params(ints[0], ints[1], ints[2], ints[3], *floats)

    def with_iters(self, iters: int) -> "Params":
        return Params(self.nx, self.ny, int(iters), self.reynolds_dim, self.density, self.accel, self.omega)


@dataclass(frozen=True)
class Params3D:
    """D3Q19 extension (include/lbm3d_hip.h; no reference counterpart)."""
    nx: int
    ny: int
    nz: int
    max_iters: int
    density: float
    accel: float
    omega: float


def channel_obstacles3d(nx: int, ny: int, nz: int) -> np.ndarray:
    """Wall planes at y = 0 and y = ny-1 (a Poiseuille channel, periodic in x and z)."""
    o = np.zeros((nz, ny, nx), np.uint8)
    o[:, 0, :] = 1
    o[:, -1, :] = 1
    return o


def read_obstacles(nx: int, ny: int, filename: str) -> "np.ndarray | None":
    """`x y 1` lines -> uint8[ny][nx] (LbmParams.hpp:92-123). None on failure."""
    data = np.zeros((ny, nx), np.uint8)
    try:
        f = open(filename, "r")
    except OSError:
        print(f"Could not read parameters from {filename}", file=sys.stderr)
        return None
    with f:
        for line in f:
            parts = line.split()
            if not parts:
                break  # reference: a line sscanf cannot parse ends the read
            try:
                x, y, o = int(parts[0]), int(parts[1]), int(parts[2])
            except (IndexError, ValueError):
                print("Malformed line: obstacle must be 1", file=sys.stderr)
                return None
            if o != 1:
                print("Malformed line: obstacle must be 1", file=sys.stderr)
                return None
            if not (0 <= x < nx and 0 <= y < ny):
                print(f"obstacle ({x},{y}) outside the {nx}x{ny} grid", file=sys.stderr)
                return None
            data[y, x] = 1
    return data


def init_cells(p: Params) -> np.ndarray:
    """Equilibrium at rest, AoS float32[ny][nx][9] (LatticeBoltzmannUtils.hpp:137-157)."""
    d = np.float32(p.density)
    w = np.array([d * np.float32(4.0) / np.float32(9.0)] + [d / np.float32(9.0)] * 4 + [d / np.float32(36.0)] * 4,
                 np.float32)
    return np.broadcast_to(w, (p.ny, p.nx, Q)).copy()


def reynolds_number(p: Params, average_velocity: float) -> float:
    viscosity = np.float32(1.0) / np.float32(6.0) * (np.float32(2.0) / np.float32(p.omega) - np.float32(1.0))
    return float(np.float32(average_velocity) * np.float32(p.reynolds_dim) / viscosity)


def macroscopic(p: Params, obstacles: np.ndarray, cells: np.ndarray):
    """Per-cell (u_x, u_y, |u|, pressure) in fp32 exactly as writeResults computes them."""
    c = cells.astype(np.float32, copy=False)
    rho = np.zeros(c.shape[:2], np.float32)
    for k in range(Q):   # sequential sum, speed order (LatticeBoltzmannUtils.hpp:249-251)
        rho = rho + c[..., k]
    ux = (((c[..., 1] + c[..., 5]) + c[..., 8]) - ((c[..., 3] + c[..., 6]) + c[..., 7])) / rho
    uy = (((c[..., 2] + c[..., 5]) + c[..., 6]) - ((c[..., 4] + c[..., 7]) + c[..., 8])) / rho
    u = np.sqrt(ux * ux + uy * uy, dtype=np.float32)
    pressure = rho * C_SQ
    ob = obstacles.astype(bool)
    ux = np.where(ob, np.float32(0), ux)
    uy = np.where(ob, np.float32(0), uy)
    u = np.where(ob, np.float32(0), u)
    pressure = np.where(ob, np.float32(p.density) * C_SQ, pressure).astype(np.float32)
    return ux, uy, u, pressure


def write_average_velocities(filename: str, av_vels) -> bool:
    """`i:\\t%.12e` per step (iostream scientific, precision 12)."""
    try:
        with open(filename, "w") as f:
            f.write("".join(f"{i}:\t{float(v):.12e}\n" for i, v in enumerate(np.asarray(av_vels, np.float32))))
        return True
    except OSError:
        return False


def write_results(filename: str, p: Params, obstacles: np.ndarray, cells: np.ndarray) -> bool:
    """final_state.dat: `ii jj u_x u_y |u| pressure obstacle`, jj outer, ii inner."""
    ux, uy, u, pr = macroscopic(p, obstacles, cells)
    jj, ii = np.meshgrid(np.arange(p.ny), np.arange(p.nx), indexing="ij")
    cols = [ii.ravel(), jj.ravel(), ux.ravel(), uy.ravel(), u.ravel(), pr.ravel(), obstacles.ravel().astype(int)]
    try:
        with open(filename, "w") as f:
            f.writelines(f"{a} {b} {c:.12e} {d:.12e} {e:.12e} {g:.12e} {h}\n"
                         for a, b, c, d, e, g, h in zip(*[col.tolist() for col in cols]))
        return True
    except OSError:
        return False


# ---- one process per GPU: rank-0 scatter / gather of sub-domain AoS blocks ----
#
# With lbm_load_cells_local / lbm_store_local (include/lbm_hip.h) a rank only
# holds its own rectangle of the lattice (16384^2 is 9.66 GB of AoS per full
# copy).  Rank 0 keeps the full-domain array the reference's loaders and .dat
# writers use (LbmRunner.cpp:67-113) and moves the blocks over a
# torch.distributed process group (gloo: host tensors).

def scatter_subdomains(full, rects, group=None):
    """Rank 0: full AoS float32[ny][nx][9]; every rank: returns its block
    full[y0:y0+h, x0:x0+w] (rects[rank], e.g. from lbm_partition)."""
    import torch
    import torch.distributed as dist
    rank = dist.get_rank(group)
    x0, y0, w, h = rects[rank]
    if rank == 0:
        for r, (rx, ry, rw, rh) in enumerate(rects):
            if r == 0:
                continue
            blk = np.ascontiguousarray(full[ry:ry + rh, rx:rx + rw], dtype=np.float32)
            dist.send(torch.from_numpy(blk), dst=r, group=group)
        return np.ascontiguousarray(full[y0:y0 + h, x0:x0 + w], dtype=np.float32)
    buf = torch.empty((h, w, 9), dtype=torch.float32)
    dist.recv(buf, src=0, group=group)
    return buf.numpy()


def gather_subdomains(block, rects, nx, ny, group=None):
    """Every rank passes its block (rects[rank]); rank 0 returns the full AoS
    float32[ny][nx][9], the others None."""
    import torch
    import torch.distributed as dist
    rank = dist.get_rank(group)
    if rank != 0:
        dist.send(torch.from_numpy(np.ascontiguousarray(block, dtype=np.float32)), dst=0, group=group)
        return None
    full = np.empty((ny, nx, 9), np.float32)
    x0, y0, w, h = rects[0]
    full[y0:y0 + h, x0:x0 + w] = block
    for r, (rx, ry, rw, rh) in enumerate(rects):
        if r == 0:
            continue
        buf = torch.empty((rh, rw, 9), dtype=torch.float32)
        dist.recv(buf, src=r, group=group)
        full[ry:ry + rh, rx:rx + rw] = buf.numpy()
    return full
