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
periodic halos as StructuredGridUtils.hpp:805-851.

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


if __name__ == "__main__":
    sys.exit(main())
