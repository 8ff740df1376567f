#!/usr/bin/env python3
"""Benchmark of the D2Q9-BGK hot path (BASELINE.json metric: MLUPS, fp32).

  python bench.py [--gpus N --steps K --warmup W] [--tile 8192x8192]
                  [--kernel auto|stream|step2|vec4|scalar] [--spl S]

One "step" = one fused lattice update of every cell (pull-stream, rebound /
BGK collision, folded acceleration, |u| reduction, halo exchange).

Workload (config.workload): BASELINE config 3, 8192x8192 fp32 cells per GPU
with deterministic synthetic obstacles (walls on the four borders plus one
full interior column at x = nx/3, mimicking obstacles_1024x1024.dat), rho 0.1,
accel 0.005, omega 1.85, equilibrium start.  For N > 1 the per-GPU tile is
fixed (weak scaling): the tiles are stacked in y, global grid 8192 x
(8192*N), one y slab per GPU (process), halos (north / south rows only) over
RCCL.  Slabs rather than the reference's 2-D partitionForIpus blocks (1x2,
2x2, 2x4, kept for config 4 below): the strip kernel walks rows, so a cut in
x leaves 4-column boundary strips that cost nearly a full strip each -- on
one GPU 4 slabs run 243 GLUPS against 192 for 2x2 blocks and 8 slabs 235
against 223 for 2x4 (profiles/r01/stream/ab_parts_weak.log).  Rank 0 at N=1 also runs BASELINE config 2 (the
reference 1024x1024 problem, 20 000 steps) and the CPU baseline.  Every N
also reports, under "aux": config 4 (the fixed 16384x16384 grid split over
all ranks: strong scaling) and config 5 (D3Q19 512^3 in z slabs over all
ranks).  Why 8192^2 per GPU is `value` although the metric also names 1024^2:
it is the HBM-roofline configuration (config 3, inputs resident in HBM, 4.8 GB
of lattice traffic per step) and the one that weak-scales to N GPUs; the
1024^2 reference problem runs on chip (resident kernel) and is reported as
aux.config2_1024x1024.

Timed region: K steps between barrier + torch.cuda.synchronize() pairs, max
over ranks.  value = all cells x K / seconds / 1e6 (whole job).

roofline: 72 algorithmic bytes per cell per LAUNCH (9 fp32 loads + 9 fp32
stores; the 1-byte obstacle mask is excluded) -- a fused launch advances
steps_per_launch time steps (the default stream kernel: 4) but moves the
lattice through HBM once -- divided by the average launch duration measured
with HIP events recorded by the library on the kernel's own stream over the
timed region (device time of the K steps / launches); peak = 8000 GB/s
(MI355X HBM3E spec).  traffic = PMC-measured HBM bytes per launch from
profiles/traffic.json (FETCH_SIZE x 2 + WRITE_SIZE, gfx950 correction) when a
profile of this workload + kernel exists, else null.  effective_gbs = 72 B x
cell updates / s (SURVEY 8(d)'s MLUPS x 72 B form), which exceeds the HBM
peak once temporal blocking pays.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
PKG = ROOT / "lbm-graphcore_amd"
for _p in (str(ROOT), str(PKG)):
    if _p not in sys.path:
        sys.path.insert(0, _p)

from lbm_amd import io as lio  # noqa: E402
from lbm_amd import native  # noqa: E402

HBM_PEAK_GBS = 8000.0
BYTES_PER_UPDATE = 72
METRIC = "MLUPS at 1024² and 8192² fp32, 1/2/4/8 MI355X; % HBM roofline"


def synthetic_obstacles(nx: int, ny: int) -> np.ndarray:
    o = np.zeros((ny, nx), np.uint8)
    o[0, :] = 1
    o[-1, :] = 1
    o[:, 0] = 1
    o[:, -1] = 1
    o[:, nx // 3] = 1
    return o


def weak_grid(n: int):
    """(rows, columns) of per-GPU tiles: y slabs (see the module docstring)."""
    return (n, 1)


def log(msg: str) -> None:
    print(msg, file=sys.stderr, flush=True)


def load_traffic(workload_key: str):
    """Per-launch HBM bytes (PMC, gfx950-corrected) from the committed profile of
    this workload + kernel, if one was recorded (tools/pmc_traffic.py)."""
    f = ROOT / "profiles" / "traffic.json"
    if not f.exists():
        return None
    try:
        d = json.loads(f.read_text())
        return d.get(workload_key, {}).get("hbm_bytes_per_launch")
    except (ValueError, OSError):
        return None


def cpu_baseline() -> dict | None:
    """The reference's own LastChance (oracle/_ref) on a bounded sample of the
    1024x1024 reference problem, single thread on this host."""
    from oracle import oracle  # checker / baseline only
    iters = 500
    gold = ROOT / "tests" / "golden" / "params"
    with tempfile.TemporaryDirectory() as wd:
        pf = Path(wd) / "bench.params"
        pf.write_text(f"1024\n1024\n{iters}\n10\n0.1\n0.01\n1.85\n")
        of = gold / "obstacles_1024x1024.dat"
        if oracle.REF_LASTCHANCE.exists():
            try:
                r = oracle.run_reference(str(pf), str(of), wd)
                secs = r["elapsed_s"]
                return {"value": round(1024 * 1024 * iters / secs / 1e6, 2), "unit": "MLUPS", "cores": 1,
                        "kind": "reference",
                        "sample": f"main/LastChance.cpp (compiled -O3 -ffp-contract=off) on the 1024x1024 "
                                  f"reference problem, first {iters} of 20000 steps, {secs:.2f} s, 1 thread"}
            except Exception as exc:  # fall back to the restatement
                log(f"reference CPU baseline failed: {exc}")
        p = lio.Params.from_file(str(pf))
        obst = lio.read_obstacles(p.nx, p.ny, str(of))
        t = time.perf_counter()
        oracle.run(p, obst)
        secs = time.perf_counter() - t
        return {"value": round(1024 * 1024 * iters / secs / 1e6, 2), "unit": "MLUPS", "cores": 1, "kind": "port",
                "sample": f"oracle/lbm_oracle.c restatement, 1024x1024 reference problem, {iters} steps, "
                          f"{secs:.2f} s, 1 thread"}


def cpu_baseline_threads() -> dict:
    """Informational all-cores CPU number ('the build's CPU restatement
    with OpenMP'): oracle_run_mt on the 1024x1024 reference problem, 60 steps, on
    OMP_NUM_THREADS threads (16 on the GPU box), lattice bitwise equal to the
    single-thread restatement."""
    from oracle import oracle  # checker / baseline only
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    gold = ROOT / "tests" / "golden" / "params"
    p = lio.Params.from_file(str(gold / "input_1024x1024.params")).with_iters(60)
    obst = lio.read_obstacles(p.nx, p.ny, str(gold / "obstacles_1024x1024.dat"))
    oracle.run_mt(p, obst, 2, threads)  # warm the thread pool
    t = time.perf_counter()
    oracle.run_mt(p, obst, 60, threads)
    secs = time.perf_counter() - t
    return {"value": round(1024 * 1024 * 60 / secs / 1e6, 1), "unit": "MLUPS", "cores": threads, "kind": "port",
            "sample": f"oracle/lbm_oracle.c oracle_run_mt (OpenMP rows), 1024x1024 reference problem, 60 steps, "
                      f"{secs:.2f} s"}


def aux_1024(kernel: int, flags: int, spl: int = 0) -> dict:
    """BASELINE config 2: the reference 1024x1024 problem, all 20 000 steps, 1 GPU."""
    gold = ROOT / "tests" / "golden" / "params"
    p = lio.Params.from_file(str(gold / "input_1024x1024.params"))
    obst = lio.read_obstacles(p.nx, p.ny, str(gold / "obstacles_1024x1024.dat"))
    with native.Engine(p, obst, devices=[0], kernel=kernel, flags=flags, steps_per_launch=spl) as e:
        e.load_cells(lio.init_cells(p))
        e.run()                      # first run: warm-up + results
        _, av = e.store()
        e.run()                      # timed re-run (device events), as LbmRunner's readTimer runs
        secs = e.last_run_seconds()
        used = e.kernel_in_use()
    cells = p.nx * p.ny
    note = ("lattice held on chip (LDS) for the whole run by the resident kernel: bound by the per-step "
            "neighbour hand-off and the collision, not by HBM" if used == "resident" else
            "lattice pair (151 MB) fits the 256 MB Infinity Cache: not an HBM-roofline number")
    return {"grid": "1024x1024", "steps": p.max_iters, "kernel": used,
            "mlups": round(cells * p.max_iters / secs / 1e6, 1),
            "ms_per_step": round(secs / p.max_iters * 1e3, 5),
            "reynolds": lio.reynolds_number(p, float(av[-1])), "note": note}


def aux_strong_16384(steps: int, rank: int, world: int, local_rank: int, dist_on: bool) -> dict:
    """BASELINE config 4: the fixed 16384x16384 grid (synthetic obstacles) over all
    ranks, RCCL halos overlapped with the interior -- whole-job MLUPS (strong
    scaling; the target is >= 6x at 8 GPUs over 1).  Split into y slabs (N x 1)
    rather than the reference's partitionForIpus blocks (1x2, 2x2, 2x4, the
    engine's default and lbm_partition's answer): emulated on one GPU, 2/4/8
    slabs ran 250/246/202 GLUPS against 200/199/182 for the blocks
    (profiles/r01/stream/ab_parts_strong.log)."""
    import torch.distributed as dist
    n = 16384
    p = lio.Params(n, n, steps, 10, 0.1, 0.005, 1.85)
    obst = synthetic_obstacles(n, n)
    kw = dict(devices=[local_rank])
    if dist_on:
        box = [native.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        kw.update(parts=world, grid=(world, 1), transport=native.TRANSPORT_RCCL, rank=rank, world=world,
                  unique_id=box[0])
    with native.Engine(p, obst, **kw) as e:
        e.init_equilibrium()
        e.run_steps(8, accelerate_first=True)
        if dist_on:
            dist.barrier()
        t0 = time.perf_counter()
        e.run_steps(steps)
        if dist_on:
            dist.barrier()
        secs = time.perf_counter() - t0
        kernel_used = e.kernel_in_use()
        rect = e.local_rects()[0]
    if dist_on:
        import torch
        t = torch.tensor([secs], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        secs = float(t[0])
    return {"grid": f"{n}x{n}", "steps": steps, "decomposition": f"{world}x1 (y slabs)",
            "sub_domain": f"{rect[2]}x{rect[3]}", "kernel": kernel_used,
            "mlups": round(n * n * steps / secs / 1e6, 1), "ms_per_step": round(secs / steps * 1e3, 4)}


def aux_d3q19(n: int, steps: int, rank: int, world: int, local_rank: int, dist_on: bool) -> dict:
    """BASELINE config 5: D3Q19 n^3 channel (body force between wall planes y = 0 and
    y = n-1), z slabs over all ranks (RCCL faces), whole-job MLUPS (strong scaling:
    the global grid is fixed).  No reference counterpart: parity pinned only by the
    CPU restatement (tests/test_d3q19.py)."""
    import torch.distributed as dist
    p = lio.Params3D(n, n, n, steps, 0.1, 0.001, 1.85)
    obst = lio.channel_obstacles3d(n, n, n)
    kw = dict(devices=[local_rank])
    if dist_on:
        box = [native.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        kw.update(transport=native.TRANSPORT_RCCL, rank=rank, world=world, unique_id=box[0])
    with native.Engine3D(p, obst, **kw) as e:
        e.init_equilibrium()
        e.run_steps(3)
        if dist_on:
            dist.barrier()
        t0 = time.perf_counter()
        e.run_steps(steps)
        if dist_on:
            dist.barrier()
        secs = time.perf_counter() - t0
        dev = e.last_run_seconds()
    if dist_on:
        import torch
        t = torch.tensor([secs, dev], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        secs, dev = float(t[0]), float(t[1])
    cells = n ** 3
    # one slab: two steps per pass (step3d_two: 60 x 8 owned of 64 x 12 loaded
    # cells per plane -> (19 x 4 B x (768/480 + 1)) / 2 = 98.8 B per update);
    # slabs: one step per launch, 152 B per update
    two = world == 1
    alg_b = 19 * 4 * (768 / 480 + 1) / 2 if two else 152
    per_gpu_gbs = alg_b * cells / world * steps / dev / 1e9
    return {"grid": f"{n}^3", "steps": steps, "decomposition": f"{world} z slabs",
            "kernel": "step3d_two (2 steps per pass)" if two else "step3d_pair (1 step per launch)",
            "mlups": round(cells * steps / secs / 1e6, 1), "ms_per_step": round(secs / steps * 1e3, 4),
            "hbm_gbs_per_gpu": round(per_gpu_gbs, 1), "hbm_frac": round(per_gpu_gbs / HBM_PEAK_GBS, 4),
            "effective_gbs_per_gpu": round(152 * cells / world * steps / dev / 1e9, 1),
            "note": f"{alg_b:.1f} algorithmic B per update (152 = 19 fp32 loads + stores per step; effective_gbs on "
                    "that basis); parity unpinned upstream (no 3-D reference)"}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--tile", default="8192x8192", help="cells per GPU, NXxNY")
    ap.add_argument("--kernel", default="auto", choices=["auto", "resident", "stream", "step2", "vec4", "scalar", "pipeline"],
                    help="stream: fused S-step register-streaming kernel; step2: fused two-step LDS kernel; "
                         "vec4/scalar: one step per launch; auto: the library's choice")
    ap.add_argument("--spl", type=int, default=0, help="stream: time steps per launch (2..4; 0 = library default)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-aux", action="store_true")
    ap.add_argument("--no-d3q19", action="store_true")
    ap.add_argument("--no-strong", action="store_true", help="skip the 16384^2 strong-scaling aux (config 4)")
    ap.add_argument("--d3q19-n", type=int, default=512, help="D3Q19 aux grid edge (BASELINE config 5: 512)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    n = world
    kernel = {"auto": native.KERNEL_AUTO, "resident": native.KERNEL_RESIDENT, "pipeline": native.KERNEL_PIPELINE, "stream": native.KERNEL_STREAM, "step2": native.KERNEL_STEP2,
              "scalar": native.KERNEL_SCALAR, "vec4": native.KERNEL_VEC4}[args.kernel]
    kflags = native.FLAG_ONE_STEP if args.kernel in ("vec4", "scalar") else 0

    import torch
    import torch.distributed as dist
    dist_on = world > 1
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(local_rank)

    tnx, tny = (int(v) for v in args.tile.lower().split("x"))
    R, C = weak_grid(n)
    nx, ny = tnx * C, tny * R
    p = lio.Params(nx, ny, args.steps, 10, 0.1, 0.005, 1.85)
    obst = synthetic_obstacles(nx, ny)

    uid = None
    if dist_on:
        box = [native.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        uid = box[0]
    eng = native.Engine(p, obst, parts=n, grid=(R, C),
                        transport=native.TRANSPORT_RCCL if dist_on else native.TRANSPORT_LOCAL,
                        rank=rank, world=world, devices=[local_rank], unique_id=uid, kernel=kernel, flags=kflags,
                        steps_per_launch=args.spl)
    eng.init_equilibrium()
    if args.warmup > 0:
        eng.run_steps(args.warmup, accelerate_first=True)

    def barrier():
        if dist_on:
            dist.barrier()

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.run_steps(args.steps, accelerate_first=False)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    dev_secs = eng.last_run_seconds()
    if dist_on:
        t = torch.tensor([elapsed, dev_secs], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, dev_secs = float(t[0]), float(t[1])
    _, av = eng.store(cells=False, n_av=args.steps)
    finite = bool(np.all(np.isfinite(av)))
    kernel_used = eng.kernel_in_use()
    steps_per_launch = eng.steps_per_launch()
    eng.close()

    total_cells = nx * ny
    value = total_cells * args.steps / elapsed / 1e6
    # a fused launch advances steps_per_launch time steps and moves the
    # lattice through HBM once: 72 algorithmic bytes per cell per launch
    launches = max(args.steps // steps_per_launch, 1)
    per_launch_s = dev_secs / launches
    cells_per_gpu = tnx * tny
    achieved = BYTES_PER_UPDATE * cells_per_gpu / per_launch_s / 1e9
    effective = achieved * steps_per_launch
    wl_key = f"{tnx}x{tny}/{kernel_used}" + (str(steps_per_launch) if kernel_used == "stream" else "")
    traffic = load_traffic(wl_key)

    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "MLUPS",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (deterministic obstacles: border walls + interior column at x=nx/3; equilibrium start)",
        "config": {"workload": f"D2Q9-BGK fused step, {tnx}x{tny} fp32 cells per GPU",
                   "global_grid": f"{nx}x{ny}", "decomposition": f"{R}x{C}",
                   "parallelism": f"{n} y slabs, one per GPU, RCCL halo exchange" if n > 1 else "single GPU",
                   "kernel": kernel_used},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "bytes_per_launch": BYTES_PER_UPDATE * cells_per_gpu,
                     "cell_updates_per_launch": steps_per_launch * cells_per_gpu,
                     "steps_per_launch": steps_per_launch,
                     "avg_launch_ms": round(per_launch_s * 1e3, 5),
                     # SURVEY 8(d) form: 72 B x cell updates / s; a fused S-step launch moves
                     # the lattice through HBM once per S updates, so this can exceed the peak
                     "effective_gbs": round(effective, 1),
                     "effective_frac": round(effective / HBM_PEAK_GBS, 4)},
        "av_vels_finite": finite,
    }
    if not args.no_aux and not args.no_strong:
        try:
            aux4 = aux_strong_16384(100, rank, world, local_rank, dist_on)
        except Exception as exc:
            aux4 = {"error": str(exc)}
        out.setdefault("aux", {})["config4_16384x16384"] = aux4
    if not args.no_aux and not args.no_d3q19:
        try:
            aux3 = aux_d3q19(args.d3q19_n, 20, rank, world, local_rank, dist_on)
        except Exception as exc:
            aux3 = {"error": str(exc)}
        out.setdefault("aux", {})["config5_d3q19"] = aux3
    if rank == 0 and n == 1:
        if not args.no_aux:
            try:
                out.setdefault("aux", {})["config2_1024x1024"] = aux_1024(kernel, kflags, args.spl)
            except Exception as exc:
                out.setdefault("aux", {})["config2_1024x1024"] = {"error": str(exc)}
        if not args.no_cpu_baseline:
            try:
                out["cpu_baseline"] = cpu_baseline()
            except Exception as exc:
                out["cpu_baseline"] = None
                log(f"cpu baseline failed: {exc}")
            try:
                out.setdefault("aux", {})["cpu_baseline_threads"] = cpu_baseline_threads()
            except Exception as exc:
                log(f"threaded cpu baseline failed: {exc}")
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
