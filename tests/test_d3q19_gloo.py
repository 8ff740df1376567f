"""D3Q19 z-slab decomposition on the CPU (gloo, world_size 2, 3 and 4).

Mirrors the engine's multi-rank D3Q19 path (lbm-graphcore_amd/csrc/lbm3d.hip):
round-robin z extents, and after every step each rank sends its top plane's
speeds 9..13 (c_z = +1, one contiguous block) up and its bottom plane's speeds
14..18 down, posted in the same order as the RCCL group (send up, send down,
receive from below, receive from above) -- the list comes from the library
(lbm3d_exchange_schedule, what the RCCL exchange posts) and is posted
untagged.  The step is the CPU restatement on
the ghosted slab; ghost-plane speeds the plan does not deliver are NaN, so a
missing or misrouted population shows up.  The gathered lattice must equal the
single-domain restatement bit for bit.  (Parity unpinned upstream: the
reference has no 3-D code.)
"""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest

from conftest import PKG, ROOT

STEPS = 5
UP = slice(9, 14)     # c_z = +1: leave through the top face
DOWN = slice(14, 19)  # c_z = -1: leave through the bottom face


def _problem():
    sys.path[:0] = [str(ROOT), str(PKG)]
    from lbm_amd import io as lio
    from oracle import oracle
    nx, ny, nz = 10, 7, 11
    p = lio.Params3D(nx, ny, nz, STEPS, 0.1, 0.003, 1.7)
    rng = np.random.default_rng(5)
    obst = lio.channel_obstacles3d(nx, ny, nz)
    obst[rng.random((nz, ny, nx)) < 0.06] = 1
    c0 = (oracle.init_cells3d(p) * (1 + 0.03 * rng.standard_normal((nz, ny, nx, 19)))).astype(np.float32)
    return p, obst, c0


def _extents(nz, world):
    n = [nz // world + (1 if i < nz % world else 0) for i in range(world)]
    z0 = [sum(n[:i]) for i in range(world)]
    return z0, n


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
        p, obst, c0 = _problem()
        z0s, nzs = _extents(p.nz, world)
        z0, n = z0s[rank], nzs[rank]
        up, down = (rank + 1) % world, (rank + world - 1) % world
        g = np.full((n + 2, p.ny, p.nx, 19), np.nan, np.float32)
        g[1:n + 1] = c0[z0:z0 + n]
        my_obst = np.ascontiguousarray(obst[z0:z0 + n])
        tots = []
        for _ in range(STEPS):
            g[0] = np.nan
            g[-1] = np.nan
            below = torch.empty((p.ny, p.nx, 5), dtype=torch.float32)
            above = torch.empty((p.ny, p.nx, 5), dtype=torch.float32)
            reqs = []
            # the engine's own posting list (lbm3d_exchange_schedule, one-step
            # face exchange), untagged: with two slabs up == down and gloo pairs
            # the two messages by order, as RCCL does
            for op, d, peer, floats in native.exchange_schedule3d(p.nx, p.ny, p.nz, world, rank, 1):
                assert peer == (up if d == 0 else down)
                assert floats == 5 * p.ny * ((p.nx + 15) // 16 * 16)  # the engine's padded speed planes
                if op == native.XFER_SEND:
                    face = g[n][..., UP] if d == 0 else g[1][..., DOWN]
                    reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(face)), dst=peer))
                else:
                    reqs.append(dist.irecv(below if d == 1 else above, src=peer))
            for r in reqs:
                r.wait()
            g[0][..., UP] = below.numpy()
            g[-1][..., DOWN] = above.numpy()
            out, tot = oracle.step3d_slab(p, g, my_obst)
            g[1:n + 1] = out
            tots.append(tot)
        t = torch.tensor(tots, dtype=torch.float64)
        all_t = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(all_t, t)
        block = torch.from_numpy(np.ascontiguousarray(g[1:n + 1]))
        if rank == 0:
            full = np.full_like(c0, np.nan)
            full[z0:z0 + n] = block.numpy()
            for src in range(1, world):
                buf = torch.empty((nzs[src], p.ny, p.nx, 19), dtype=torch.float32)
                dist.recv(buf, src=src)
                full[z0s[src]:z0s[src] + nzs[src]] = buf.numpy()
            result_q.put((full, np.sum(np.stack([a.numpy() for a in all_t]), axis=0)))
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


@pytest.mark.parametrize("world", [2, 3, 4])
def test_gloo_d3q19_slabs_match_single_domain(world):
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
    p, obst, c0 = _problem()
    ref, ref_av = oracle.run3d(p, obst, STEPS, c0)
    assert not np.isnan(full).any()
    assert np.array_equal(full, ref)
    np.testing.assert_allclose(tot / oracle.free_cells3d(p, obst), ref_av, rtol=1e-5)
