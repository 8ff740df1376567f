"""Multi-rank CPU restatement of the exchange the DEFAULT (fused) path uses.

The fused launches (stream kernel, S steps per launch) exchange the S
outermost rows / columns of every sub-domain with ALL nine populations ("WG"
halo: S x len strips for the four sides, S x S blocks for the corners) once
per launch, and RCCL matches the messages between two ranks purely by posting
order: the engine posts, for d = E, N, W, S, NE, NW, SW, SE, the send of the
strip leaving through d to the neighbour there, then the receive of ghost
side OPP(d) from the neighbour there (lbm_engine.hip exchange_posts, posted
by exchange() in one ncclGroupStart/End block).  Here every rank posts the
same list with gloo isend /
irecv and NO tags (one default tag: messages to one peer match in order),
then advances S steps on its ghosted block with the CPU oracle (the ring
shrinks by one cell per step), and the gathered lattice must equal the
single-domain oracle bit for bit.  The posts come from the library itself
(lbm_exchange_schedule, the list exchange() iterates), not from a Python
restatement of the order.  Extent-2 dimensions (1x2, 2x1, 2x2, 2x4)
send several messages to the same peer per exchange, which is exactly where
order matching matters; 8x1 and 2x4 are the bench's two 8-GPU layouts.
Reference side of the contract: the per-step stitched halos of
main/LbmAoS.cpp:151-160 and the periodic halo slices of
main/include/StructuredGridUtils.hpp:805-851.

The same workers also check the rank-0 scatter / gather helpers
(lbm_amd.io.scatter_subdomains / gather_subdomains) that pair with
lbm_load_cells_local / lbm_store_local.
"""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest

from conftest import PKG, ROOT

LAUNCHES = 2  # fused launches per S (S*LAUNCHES steps)
DIRS = [(1, 0), (0, 1), (-1, 0), (0, -1), (1, 1), (-1, 1), (-1, -1), (1, -1)]  # E N W S NE NW SW SE
OPP = [2, 3, 0, 1, 6, 7, 4, 5]


def _problem():
    sys.path[:0] = [str(ROOT), str(PKG)]
    from lbm_amd import io as lio
    nx, ny = 48, 72
    p = lio.Params(nx, ny, 8, 10, 0.1, 0.02, 1.7)
    rng = np.random.default_rng(23)
    obst = (rng.random((ny, nx)) < 0.04).astype(np.uint8)
    obst[0, :] = 1
    obst[10:40, 17] = 1
    cells0 = (lio.init_cells(p) * (1 + 0.03 * rng.standard_normal((ny, nx, 9)))).astype(np.float32)
    return p, obst, cells0


def _edge(g, S, w, h, dx, dy):
    """Index ranges (ghosted block with ring S) of the S outermost cells on side (dx, dy)."""
    ys = slice(S, S + h) if dy == 0 else (slice(S + h - S, S + h) if dy > 0 else slice(S, 2 * S))
    xs = slice(S, S + w) if dx == 0 else (slice(S + w - S, S + w) if dx > 0 else slice(S, 2 * S))
    return ys, xs


def _ghost(S, w, h, dx, dy):
    """Index ranges of the ghost region on side (dx, dy)."""
    ys = slice(S, S + h) if dy == 0 else (slice(S + h, 2 * S + h) if dy > 0 else slice(0, S))
    xs = slice(S, S + w) if dx == 0 else (slice(S + w, 2 * S + w) if dx > 0 else slice(0, S))
    return ys, xs


def _pack(g, ys, xs, d):
    """The engine's WG message layout: [9][S][len] for sides ((strip column, row)
    for E/W, (strip row, column) for N/S), [9][S][S] (strip row, strip column) for corners."""
    blk = g[ys, xs]                      # [rows][cols][9]
    if d in (0, 2):                      # E / W: [9][col][row]
        return np.ascontiguousarray(blk.transpose(2, 1, 0))
    return np.ascontiguousarray(blk.transpose(2, 0, 1))  # N / S / corners: [9][row][col]


def _unpack(msg, d):
    if d in (0, 2):
        return msg.transpose(2, 1, 0)
    return msg.transpose(1, 2, 0)


def _step_region(oracle, p, src, obst_ext, gy0):
    """One oracle step of every cell of src's interior (src: (H+2, W+2, 9));
    obst_ext: (H, W) obstacles of the output cells; gy0: global row of output
    row 0 (mod ny).  Row by row, so the accelerated row is found wherever the
    periodic images put it."""
    H, W = src.shape[0] - 2, src.shape[1] - 2
    out = np.empty((H, W, 9), np.float32)
    pp = type(p)(W, 1, p.max_iters, p.reynolds_dim, p.density, p.accel, p.omega)
    for r in range(H):
        acc = 0 if (gy0 + r) % p.ny == p.ny - 2 else -1
        out[r], _ = oracle.step_ghosted(pp, src[r:r + 3], obst_ext[r:r + 1], acc)
    return out


def _owned_tot(oracle, p, src, obst, gy0, S):
    """|u| sum over the owned cells only (for av_vels), from the ghosted input."""
    h, w = obst.shape
    sub = src[S - 1:S + h + 1, S - 1:S + w + 1]
    tot = np.float32(0)
    pp = type(p)(w, 1, p.max_iters, p.reynolds_dim, p.density, p.accel, p.omega)
    for r in range(h):
        acc = 0 if (gy0 + r) % p.ny == p.ny - 2 else -1
        _, t = oracle.step_ghosted(pp, sub[r:r + 3], obst[r:r + 1], acc)
        tot = np.float32(tot + np.float32(t))
    return float(tot)


def _worker(rank, world, grid, port, result_q):
    sys.path[:0] = [str(ROOT), str(PKG)]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    from lbm_amd import io as lio
    from lbm_amd import native
    from oracle import oracle
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p, obst, cells0 = _problem()
        R, C, rects = native.partition(p.nx, p.ny, world, *grid)
        assert (R, C) == grid
        x0, y0, w, h = rects[rank]
        cells_acc = cells0.copy()
        oracle.accelerate(p, cells_acc, obst)
        # rank 0 scatters the blocks (lbm_load_cells_local's host side)
        own = lio.scatter_subdomains(cells_acc if rank == 0 else None, rects)
        assert np.array_equal(own, cells_acc[y0:y0 + h, x0:x0 + w])
        results = {}
        for S in (2, 3, 4):
            assert w >= 2 * S or C == 1
            assert h >= 2 * S or R == 1
            blk = own.copy()
            tots = []
            # obstacles of the block and its S-ring (periodic images)
            ys_g = (np.arange(y0 - S, y0 + h + S) % p.ny)[:, None]
            xs_g = (np.arange(x0 - S, x0 + w + S) % p.nx)[None, :]
            obst_ring = obst[ys_g, xs_g]
            for _ in range(LAUNCHES):
                g = np.full((h + 2 * S, w + 2 * S, 9), np.nan, np.float32)
                g[S:S + h, S:S + w] = blk
                reqs, recvs = [], []
                # the engine's own posting list (lbm_exchange_schedule = what
                # exchange() posts inside one ncclGroupStart/End), no tags
                for op, d, peer, floats in native.exchange_schedule(p.nx, p.ny, world, rank, native.HALO_WG, S,
                                                                    R, C):
                    dx, dy = DIRS[d]
                    if op == native.XFER_SELF:   # periodic wrap inside this block: the image in place
                        assert peer == rank
                        gys, gxs = _ghost(S, w, h, -dx, -dy)
                        eys, exs = _edge(g, S, w, h, dx, dy)
                        g[gys, gxs] = g[eys, exs]
                    elif op == native.XFER_SEND:
                        eys, exs = _edge(g, S, w, h, dx, dy)
                        msg = _pack(g, eys, exs, d)
                        assert msg.size == floats, (d, msg.shape, floats)
                        reqs.append(dist.isend(torch.from_numpy(msg), dst=peer))
                    else:                        # ghost side d, the neighbour's strip of direction OPP(d)
                        gys, gxs = _ghost(S, w, h, dx, dy)
                        shape = _pack(g, gys, gxs, OPP[d]).shape
                        assert int(np.prod(shape)) == floats, (d, shape, floats)
                        buf = torch.empty(shape, dtype=torch.float32)
                        recvs.append((gys, gxs, OPP[d], buf))
                        reqs.append(dist.irecv(buf, src=peer))
                for r_ in reqs:
                    r_.wait()
                for gys, gxs, d, buf in recvs:
                    g[gys, gxs] = _unpack(buf.numpy(), d)
                assert not np.isnan(g).any(), "ghost ring incomplete"
                # S steps, the valid region shrinking by one cell per step
                cur = g
                for i in range(1, S + 1):
                    r_in, r_out = S - i + 1, S - i   # ring widths of the input / output
                    tots.append(_owned_tot(oracle, p, cur, obst[y0:y0 + h, x0:x0 + w], y0, r_in))
                    ob = obst_ring[S - r_out:S + h + r_out, S - r_out:S + w + r_out]
                    cur = _step_region(oracle, p, cur, ob, (y0 - r_out) % p.ny)
                blk = cur
            results[S] = (blk, np.array(tots, np.float64))
        # gather every S's lattice on rank 0 (lbm_store_local's host side)
        out = {}
        for S, (blk, tots) in results.items():
            full = lio.gather_subdomains(blk, rects, p.nx, p.ny)
            t = torch.tensor(tots)
            all_t = [torch.zeros_like(t) for _ in range(world)]
            dist.all_gather(all_t, t)
            if rank == 0:
                out[S] = (full, np.sum(np.stack([a.numpy() for a in all_t]), axis=0))
        if rank == 0:
            result_q.put(out)
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("grid", [(1, 2), (2, 1), (2, 2), (2, 4), (8, 1)], ids=lambda g: f"{g[0]}x{g[1]}")
def test_wg_exchange_in_order_matches_single_domain(grid):
    import torch.multiprocessing as mp
    from oracle import oracle
    world = grid[0] * grid[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, grid, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    out = q.get(timeout=300)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    p, obst, cells0 = _problem()
    free = oracle.free_cells(p, obst)
    for S, (full, tot) in out.items():
        steps = S * LAUNCHES
        ref, ref_av = oracle.run(p, obst, steps, cells0)
        assert not np.isnan(full).any()
        assert np.array_equal(full, ref), f"S={S}"
        np.testing.assert_allclose(tot / free, ref_av, rtol=1e-5)
