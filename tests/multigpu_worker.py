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
periodic halos as StructuredGridUtils.hpp:805-851.  Then config 4's block
decomposition (run_config4) and the D3Q19 z slabs (run_case3d): three-step
passes with a three-plane RCCL exchange per pass.  case_list() is the plan.

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


def case_list(world: int) -> dict:
    """What a world of `world` ranks runs (tests/test_multigpu_plan.py checks on
    the CPU that at world 8 it covers BASELINE config 4's 2x4 blocks and config
    5's 8 z slabs):
      grids2d   2048^2, bitwise vs the oracle, on the reference rule and on
                world x 1 slabs, 13 and 16 steps;
      config4   config 4's decomposition (16384^2 over `world` ranks by the
                reference rule: 2x4 blocks of 4096 x 8192 at world 8) at a
                quarter of the height -- 16384 x 4096, the same R x C grid and
                block width -- in tolerance mode, the driver's plan (2 x 10
                steps); every rank compares its own block bitwise with a
                single-domain run of the same library on its own GPU;
      d3q19     `world` z slabs of 8 planes (config 5's 8 slabs at world 8)."""
    R4, C4, _ = native.partition(16384, 16384, world)
    return {"grids2d": {"n": 2048, "grids": [(0, 0), (world, 1)], "steps": [13, 16]},
            "config4": {"nx": 16384, "ny": 4096, "grid": (R4, C4), "steps": 20},
            "d3q19": {"nx": 40, "ny": 22, "nz": 8 * world, "slabs": world}}


def main() -> int:
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    plan = case_list(world)
    n = plan["grids2d"]["n"]
    rng = np.random.default_rng(77)
    obst = np.zeros((n, n), np.uint8)
    obst[0, :] = obst[-1, :] = 1
    obst[:, n // 3] = 1
    obst[rng.random((n, n)) < 0.02] = 1
    cells0 = (lio.init_cells(lio.Params(n, n, 1, 10, 0.1, 0.005, 1.85)) *
              (1 + 0.02 * rng.standard_normal((n, n, 9)))).astype(np.float32)
    out = {}
    for steps in plan["grids2d"]["steps"]:
        run_case(rank, world, n, steps, obst, cells0, out, plan["grids2d"]["grids"])
    run_config4(rank, world, plan["config4"], out)
    run_case3d(rank, world, plan["d3q19"], out)
    if rank == 0:
        Path(sys.argv[1]).write_text(json.dumps(out))
    dist.barrier()
    dist.destroy_process_group()
    return 0


def run_config4(rank, world, c, out):
    """Config 4's R x C blocks over RCCL (tolerance, 2 x 10 steps) against a
    single-domain engine on this rank's GPU: each rank compares its own block;
    the verdicts are gathered over gloo."""
    import torch.distributed as dist
    nx, ny, steps = c["nx"], c["ny"], c["steps"]
    p = lio.Params(nx, ny, steps, 10, 0.1, 0.005, 1.85)
    obst = np.zeros((ny, nx), np.uint8)
    obst[0, :] = obst[-1, :] = 1
    obst[:, nx // 3] = 1
    R, C, rects = native.partition(nx, ny, world, *c["grid"])
    x0, y0, w, h = rects[rank]
    box = [native.rccl_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(box, src=0)
    with native.Engine(p, obst, parts=world, grid=c["grid"], transport=native.TRANSPORT_RCCL, rank=rank,
                       world=world, devices=[rank], unique_id=box[0], flags=native.FLAG_TOLERANCE) as e:
        e.init_equilibrium()
        e.run_steps(steps, accelerate_first=True)
        stats = e.run_stats()
        blocks, _ = e.store_local(n_av=steps)
    with native.Engine(p, obst, devices=[rank], flags=native.FLAG_TOLERANCE) as e1:
        e1.init_equilibrium()
        e1.run_steps(steps, accelerate_first=True)
        ref, _ = e1.store(n_av=steps)
    mine = {"bitwise": bool(np.array_equal(blocks[0], ref[y0:y0 + h, x0:x0 + w])), "launches": list(stats)}
    allv = [None] * world
    dist.all_gather_object(allv, mine)
    if rank == 0:
        out[f"config4/{R}x{C}/{nx}x{ny}/tolerance/{steps}"] = {
            "bitwise": all(v["bitwise"] for v in allv), "ranks_failed": [r for r, v in enumerate(allv) if not v["bitwise"]],
            "launches": allv[0]["launches"], "av_rel": 0.0}


def run_case(rank, world, n, steps, obst, cells0, out, grids):
    import torch.distributed as dist
    p = lio.Params(n, n, steps, 10, 0.1, 0.005, 1.85)
    ref = ref_av = None
    if rank == 0:
        from oracle import oracle  # the checker
        ref, ref_av = oracle.run(p, obst, steps, cells0)
    for grid in grids:
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


def run_case3d(rank, world, c, out):
    """D3Q19 z slabs over RCCL (one slab of 8 planes per rank): three-step
    passes with their three-plane exchange between real devices -- bitwise
    collision (LBM3D_THREE=1) 10 steps = three passes + one one-step launch,
    compared with the CPU restatement; tolerance collision (three-step passes
    by default) 9 steps, compared with one slab of the same library and mode
    on rank 0's GPU.  Each rank stores its own slab; summed over gloo."""
    import torch
    import torch.distributed as dist
    from oracle import oracle  # the checker (initial state, reference lattice)
    nx, ny, nz = c["nx"], c["ny"], c["nz"]
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
            assert len(e.local_slabs()) == 1 and world == c["slabs"]
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
