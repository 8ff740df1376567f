#!/usr/bin/env python3
"""Two-process RCCL transport check: world 2, one sub-domain per process,
lattice gathered and compared bitwise against the CPU oracle.

  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29555 tools/rccl_pair_check.py [--grid 1x2] [--same-device]

--same-device puts both ranks on device 0 (only to probe whether RCCL
accepts it on a one-GPU box).
"""
from __future__ import annotations

import argparse
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "lbm-graphcore_amd")]

from lbm_amd import io as lio  # noqa: E402
from lbm_amd import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", default="1x2")
    ap.add_argument("--same-device", action="store_true")
    ap.add_argument("--steps", type=int, default=17)
    a = ap.parse_args()
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    dist.init_process_group("gloo")
    R, C = (int(v) for v in a.grid.split("x"))
    gold = ROOT / "tests" / "golden" / "params"
    p = lio.Params.from_file(str(gold / "input_128x256.params")).with_iters(a.steps)
    obst = lio.read_obstacles(p.nx, p.ny, str(gold / "obstacles_128x256.dat"))
    box = [native.rccl_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(box, src=0)
    dev = 0 if a.same_device else local
    with native.Engine(p, obst, parts=world, grid=(R, C), transport=native.TRANSPORT_RCCL, rank=rank,
                       world=world, devices=[dev], unique_id=box[0]) as e:
        e.load_cells(lio.init_cells(p))
        e.run()
        cells, av = e.store()
        (x0, y0, w, h), = e.local_rects()
    import torch
    mine = torch.from_numpy(np.ascontiguousarray(cells[y0:y0 + h, x0:x0 + w]))
    meta = [None] * world
    dist.all_gather_object(meta, (x0, y0, w, h, mine.numpy()))
    if rank == 0:
        from oracle import oracle
        full = np.full_like(cells, np.nan)
        for (sx, sy, sw, sh, blk) in meta:
            full[sy:sy + sh, sx:sx + sw] = blk
        ref, ref_av = oracle.run(p, obst, a.steps, lio.init_cells(p))
        ok = np.array_equal(full, ref)
        av_ok = np.allclose(av, ref_av, rtol=1e-5)
        print(f"RCCL world={world} grid={a.grid}: lattice bitwise={ok} av_vels close={av_ok}", flush=True)
        if not (ok and av_ok):
            sys.exit(1)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
