"""One rank of tests/test_multigpu.py (started as a fresh process per GPU; the
parent never initialises HIP).  RCCL-transport engine with the fused stream
kernel (LP form, S = 6) on a 2048^2 problem (random obstacles, perturbed
start), 13 steps = two fused launches + a one-step remainder and 16 steps =
two fused launches + a fused 4-step remainder (its halo through RCCL in the
innermost ring), per-rank load/store of the
rank's own block; rank 0 gathers the blocks over gloo and compares the
lattice bitwise with the CPU oracle (LastChance.cpp:192-266 restated).
Decompositions: the reference partitionForIpus rule
(StructuredGridUtils.hpp:498-522; 2x4 for 8 ranks) and world x 1 slabs;
periodic halos as StructuredGridUtils.hpp:805-851.  Then the D3Q19 z slabs
(run_case3d): three-step passes with a three-plane RCCL exchange per pass.

usage: RANK=r WORLD_SIZE=n MASTER_ADDR=127.0.0.1 MASTER_PORT=p python multigpu_worker.py OUT.json
"""
from __future__ import annotations

import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "lbm-graphcore_amd")]

from lbm_amd import io as lio  # noqa: E402
from lbm_amd import native  # noqa: E402


def main() -> int:
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 2048
    rng = np.random.default_rng(77)
    obst = np.zeros((n, n), np.uint8)
    obst[0, :] = obst[-1, :] = 1
    obst[:, n // 3] = 1
    obst[rng.random((n, n)) < 0.02] = 1
    cells0 = (lio.init_cells(lio.Params(n, n, 1, 10, 0.1, 0.005, 1.85)) *
              (1 + 0.02 * rng.standard_normal((n, n, 9)))).astype(np.float32)
    out = {}
    for steps in (13, 16):
        run_case(rank, world, n, steps, obst, cells0, out)
    run_case3d(rank, world, out)
    if rank == 0:
        Path(sys.argv[1]).write_text(json.dumps(out))
    dist.barrier()
    dist.destroy_process_group()
    return 0


def run_case(rank, world, n, steps, obst, cells0, out):
    import torch.distributed as dist
    p = lio.Params(n, n, steps, 10, 0.1, 0.005, 1.85)
    ref = ref_av = None
    if rank == 0:
        from oracle import oracle  # the checker
        ref, ref_av = oracle.run(p, obst, steps, cells0)
    for grid in ((0, 0), (world, 1)):
        R, C, rects = native.partition(n, n, world, *grid)
        box = [native.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        with native.Engine(p, obst, parts=world, grid=grid, transport=native.TRANSPORT_RCCL, rank=rank, world=world,
                           devices=[rank], unique_id=box[0], kernel=native.KERNEL_STREAM) as e:
            assert e.local_rects() == [tuple(rects[rank])]
            x0, y0, w, h = rects[rank]
            e.load_cells_local([cells0[y0:y0 + h, x0:x0 + w]])
            e.run_steps(steps, accelerate_first=True)
            stats = e.run_stats()
            blocks, av = e.store_local(n_av=steps)
        full = lio.gather_subdomains(blocks[0], rects, n, n)
        if rank == 0:
            out[f"{R}x{C}/{steps}"] = {"bitwise": bool(np.array_equal(full, ref)), "bad": int(np.sum(full != ref)),
                                       "launches": list(stats),
                                       "av_rel": float(np.max(np.abs(av - ref_av) / np.abs(ref_av)))}


def run_case3d(rank, world, out):
    """D3Q19 z slabs over RCCL (one slab of 8 planes per rank): three-step
    passes with their three-plane exchange between real devices -- bitwise
    collision (LBM3D_THREE=1) 10 steps = three passes + one one-step launch,
    compared with the CPU restatement; tolerance collision (three-step passes
    by default) 9 steps, compared with one slab of the same library and mode
    on rank 0's GPU.  Each rank stores its own slab; summed over gloo."""
    import torch
    import torch.distributed as dist
    from oracle import oracle  # the checker (initial state, reference lattice)
    nx, ny, nz = 40, 22, 8 * world
    p = lio.Params3D(nx, ny, nz, 0, 0.1, 0.002, 1.7)
    rng = np.random.default_rng(5)
    obst = lio.channel_obstacles3d(nx, ny, nz)
    obst[rng.random((nz, ny, nx)) < 0.05] = 1
    c0 = (oracle.init_cells3d(p) * (1 + 0.02 * rng.standard_normal((nz, ny, nx, 19)))).astype(np.float32)
    os.environ["LBM_DEBUG_KNOBS"] = "1"
    os.environ["LBM3D_THREE"] = "1"
    for flags, steps in ((0, 10), (native.FLAG_TOLERANCE, 9)):
        box = [native.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        with native.Engine3D(p, obst, transport=native.TRANSPORT_RCCL, rank=rank, world=world, devices=[rank],
                             unique_id=box[0], flags=flags) as e:
            e.load_cells(c0)
            e.run_steps(steps)
            cells, av = e.store(n_av=steps)
        t = torch.from_numpy(cells)
        dist.all_reduce(t)  # every rank filled only its own slab
        full = t.numpy()
        if rank == 0:
            if flags == 0:
                ref, ref_av = oracle.run3d(p, obst, steps, c0)
            else:
                with native.Engine3D(p, obst, devices=[0], flags=flags) as e1:
                    e1.load_cells(c0)
                    e1.run_steps(steps)
                    ref, ref_av = e1.store(n_av=steps)
            out[f"d3q19/{world}slabs/{'tolerance' if flags else 'bitwise'}/{steps}"] = {
                "bitwise": bool(np.array_equal(full, ref)), "bad": int(np.sum(full != ref)),
                "av_rel": float(np.max(np.abs(av - ref_av) / np.abs(ref_av)))}
    del os.environ["LBM3D_THREE"]


if __name__ == "__main__":
    sys.exit(main())
