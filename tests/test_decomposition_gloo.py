"""Multi-rank decomposition on the CPU (gloo, world_size 2 and 4).

Each rank owns the sub-domain the library's own partition rule assigns it
(lbm_partition, StructuredGridUtils.hpp:472-561 semantics) and exchanges a
one-cell halo every step following the library's own halo plan
(lbm_halo_plan: which populations leave through which side) and the
engine's own ordered posting list (lbm_exchange_schedule, W1 format: the
sends and receives exchange() posts in one RCCL group), untagged, so gloo
pairs them by order exactly as RCCL does.  The step itself is the CPU
oracle on the ghosted block.  Ghost planes NOT covered by the plan are
poisoned with NaN, so a missing population would show up.  After N steps the
gathered lattice must equal the single-domain oracle bit for bit.
"""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest

from conftest import PKG, ROOT

STEPS = 6
OPP = [2, 3, 0, 1, 6, 7, 4, 5]   # E N W S NE NW SW SE -> opposite side


def _problem():
    sys.path[:0] = [str(ROOT), str(PKG)]
    from lbm_amd import io as lio
    nx, ny = 40, 26
    p = lio.Params(nx, ny, STEPS, 10, 0.1, 0.02, 1.7)
    obst = np.zeros((ny, nx), np.uint8)
    obst[0, :] = 1
    obst[:, 0] = 1
    obst[6:20, 13] = 1
    rng = np.random.default_rng(11)
    cells0 = (lio.init_cells(p) * (1 + 0.03 * rng.standard_normal((ny, nx, 9)))).astype(np.float32)
    return p, obst, cells0


def _ranges(dx, dy, w, h, ghost):
    """Index ranges into the (h+2, w+2) ghosted block for the edge (ghost=False)
    or the ghost region (ghost=True) on side (dx, dy)."""
    def one(dv, n):
        if dv == 0:
            return slice(1, n + 1)
        if ghost:
            return slice(n + 1, n + 2) if dv > 0 else slice(0, 1)
        return slice(n, n + 1) if dv > 0 else slice(1, 2)
    return one(dy, h), one(dx, w)


def _worker(rank, world, port, result_q):
    sys.path[:0] = [str(ROOT), str(PKG)]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    from lbm_amd import native
    from oracle import oracle
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p, obst, cells0 = _problem()
        R, C, rects = native.partition(p.nx, p.ny, world)
        plan = native.halo_plan()
        x0, y0, w, h = rects[rank]

        # the one-time accelerate is pointwise on row ny-2 (LastChance.cpp:161-183):
        # apply it to the initial state, then decompose
        cells_acc = cells0.copy()
        oracle.accelerate(p, cells_acc, obst)
        g = np.full((h + 2, w + 2, 9), np.nan, np.float32)
        g[1:h + 1, 1:w + 1] = cells_acc[y0:y0 + h, x0:x0 + w]
        my_obst = np.ascontiguousarray(obst[y0:y0 + h, x0:x0 + w])
        accel_row = (p.ny - 2) - y0 if y0 <= p.ny - 2 < y0 + h else -1

        tots = []
        for _ in range(STEPS):
            g[0, :, :] = np.nan
            g[-1, :, :] = np.nan
            g[:, 0, :] = np.nan
            g[:, -1, :] = np.nan
            reqs, bufs = [], []
            # the engine's own posting list for one-step launches (W1 halo:
            # lbm_exchange_schedule, what exchange() posts in one RCCL group),
            # in that order and with no tags: messages to one peer match by order
            for op, d, peer, floats in native.exchange_schedule(p.nx, p.ny, world, rank, native.HALO_W1):
                dx, dy, planes = plan[d]
                if op == native.XFER_SELF:   # periodic wrap inside this block
                    assert peer == rank
                    ys, xs = _ranges(dx, dy, w, h, False)
                    gy, gx = _ranges(-dx, -dy, w, h, True)
                    sub = g[gy, gx]
                    sub[..., planes] = g[ys, xs][..., planes]
                    g[gy, gx] = sub
                elif op == native.XFER_SEND:  # populations leaving through side d
                    ys, xs = _ranges(dx, dy, w, h, False)
                    data = np.ascontiguousarray(g[ys, xs][..., planes])
                    assert data.size == floats
                    reqs.append(dist.isend(torch.from_numpy(data), dst=peer))
                else:                         # ghost side d: the neighbour's populations leaving through OPP(d)
                    odx, ody, oplanes = plan[OPP[d]]
                    ys, xs = _ranges(dx, dy, w, h, True)
                    shape = g[ys, xs][..., oplanes].shape
                    assert int(np.prod(shape)) == floats
                    buf = torch.empty(shape, dtype=torch.float32)
                    bufs.append((ys, xs, oplanes, buf))
                    reqs.append(dist.irecv(buf, src=peer))
            for r in reqs:
                r.wait()
            for ys, xs, planes, buf in bufs:
                sub = g[ys, xs]
                sub[..., planes] = buf.numpy()
                g[ys, xs] = sub
            pp = type(p)(w, h, p.max_iters, p.reynolds_dim, p.density, p.accel, p.omega)
            out, tot = oracle.step_ghosted(pp, g, my_obst, accel_row)
            g[1:h + 1, 1:w + 1] = out
            tots.append(tot)
        # gather
        block = torch.from_numpy(np.ascontiguousarray(g[1:h + 1, 1:w + 1]))
        sizes = [torch.zeros(4, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(sizes, torch.tensor([x0, y0, w, h]))
        t = torch.tensor(tots, dtype=torch.float64)
        all_t = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(all_t, t)
        if rank == 0:
            full = np.full_like(cells0, np.nan)
            full[y0:y0 + h, x0:x0 + w] = block.numpy()
            for src in range(1, world):
                sx, sy, sw, sh = (int(v) for v in sizes[src])
                buf = torch.empty((sh, sw, 9), dtype=torch.float32)
                dist.recv(buf, src=src)
                full[sy:sy + sh, sx:sx + sw] = buf.numpy()
            tot = np.sum(np.stack([a.numpy() for a in all_t]), axis=0)
            result_q.put((full, tot))
        else:
            dist.send(block.contiguous(), dst=0)
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("world", [2, 4, 8])
def test_gloo_decomposition_matches_single_domain(world):
    import torch.multiprocessing as mp
    from oracle import oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    full, tot = q.get(timeout=240)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    p, obst, cells0 = _problem()
    ref, ref_av = oracle.run(p, obst, STEPS, cells0)
    assert not np.isnan(full).any()
    assert np.array_equal(full, ref)
    free = oracle.free_cells(p, obst)
    np.testing.assert_allclose(tot / free, ref_av, rtol=1e-5)
