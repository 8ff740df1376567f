#!/usr/bin/env python3
"""Benchmark of the D2Q9-BGK hot path (BASELINE.json metric: MLUPS, fp32).

  python bench.py [--gpus N --steps K --warmup W] [--tile 8192x8192]
                  [--kernel auto|stream|step2|vec4|scalar] [--spl S]
                  [--numerics tolerance|bitwise]

Numerics: `value` is measured with the collision
--numerics names -- tolerance (default: LBM_FLAG_TOLERANCE, IEEE fp32 with one
reciprocal of rho per cell, within the tolerance the line states, north_star's
"within a stated fp32 tolerance") or bitwise (every population identical to
the reference arithmetic); the other one runs the same workload in aux.
Steps per launch: the S that finishes K steps soonest by the measured launch
times (pick_spl over calibrate_launch_ms: every S timed on the box at bench
start, untimed; a remainder of >= 2 steps is one fused launch), reported in
launches.plan.

One "step" = one fused lattice update of every cell (pull-stream, rebound /
BGK collision, folded acceleration, |u| reduction, halo exchange).

Workload (config.workload): BASELINE config 3, 8192x8192 fp32 cells per GPU
with deterministic synthetic obstacles (walls on the four borders plus one
full interior column at x = nx/3, mimicking obstacles_1024x1024.dat), rho 0.1,
accel 0.005, omega 1.85, equilibrium start.  For N > 1 the per-GPU tile is
fixed (weak scaling) and the tiles are arranged by the reference's
partitionForIpus rule (StructuredGridUtils.hpp:498-522: 1x2, 2x2, 2x4 for a
square tile; rank = row*cols + col), one sub-domain per GPU (process), halos
over RCCL -- the 2-D blocks north_star names.  aux.weak_slabs runs the same
per-GPU tile as N x 1 y slabs (north/south halos only) for comparison.
Rank 0 at N=1 also runs BASELINE config 2 (the reference 1024x1024 problem,
20 000 steps) and the CPU baselines.  Every N also reports, under "aux":
config 4 (the fixed 16384x16384 grid split over all ranks by the reference
rule; strong scaling) and the same as y slabs (config4_slabs, N > 1), and
config 5 (D3Q19 512^3 in z slabs over all ranks).  Why 8192^2 per GPU is
`value` although the metric also names 1024^2: it is the HBM-roofline
configuration (config 3, inputs resident in HBM, 4.8 GB of lattice traffic
per step) and the one that weak-scales to N GPUs; the 1024^2 reference
problem runs on chip (resident kernel) and is reported as aux.config2_1024x1024.

Settling: the GPU ramps its clock for the first ~20-30 ms of back-to-back
work (tools/settle_probe.py: a 20-step run right after a 5-step warm-up took
1.38 ms per launch, the same run settled 1.20), so after the W warm-up steps
the bench runs untimed "settle" steps worth >= 0.3 s of device time (the same
count on every rank) and reports them in the JSON ("settle").

Timed region: K steps between barrier + torch.cuda.synchronize() pairs, max
over ranks.  value = all cells x K / seconds / 1e6 (whole job).

roofline: 72 algorithmic bytes per cell per LAUNCH (9 fp32 loads + 9 fp32
stores; the 1-byte obstacle mask is excluded) -- a fused launch advances
steps_per_launch time steps (S = 10 for the tolerance value at K = 20 or 1000)
but moves the lattice through HBM once -- divided by the average launch duration measured
with HIP events recorded by the library on the kernel's own stream over the
timed region (device time of the K steps / launches); peak = 8000 GB/s
(MI355X HBM3E spec).  traffic = PMC-measured HBM bytes per launch from
profiles/traffic.json (FETCH_SIZE x 2 + WRITE_SIZE, gfx950 correction) when a
profile of this workload + kernel exists, else null.  effective_gbs = 72 B x
cell updates / s (SURVEY 8(d)'s MLUPS x 72 B form), which exceeds the HBM
peak once temporal blocking pays.  roofline.valu = VALU instructions per
launch and the VALU pipe's busy fraction from the SQ pass of the same profile
(tools/pmc_traffic.py --sq).  roofline.device_copy: a device copy of one
lattice's bytes timed live on this GPU (context; never the
peak).  roofline.bound: "hbm" when frac or
frac_counter_bytes (the PMC bytes over the same launch time) reaches 0.75,
"valu" when frac_valu_issue (VALU busy in quad-cycle units) does -- the larger
wins -- and "latency" when none does (the launch waits on loads, LDS and
dependency chains rather than saturating either pipe).

cpu_baseline: the reference's main/LbmCpu.cpp as committed (north_star: "next
to LbmCpu.cpp timed on the same box's host cores"), built from its source by
oracle/Makefile, on the 128x128 reference problem (all 40 000 steps, one
thread: it has no OpenMP pragmas), timed by its own "Total compute time".  It
is cost-only: its live kernel fails check.py upstream.
aux.cpu_config1_128x128 is the config-1 plumbing record (LastChance.cpp, the
reference's correct CPU path, full 128x128 run gated by check.py against the
reference's check/ fixtures); aux.cpu_lastchance_1024x1024 a bounded sample
of the 1024x1024 problem; aux.cpu_baseline_threads the restatement on every
host core.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import threading
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


def weak_grid(n: int, tnx: int, tny: int, slabs: bool = False):
    """(rows, columns) of per-GPU tiles: the reference rule for a tile-shaped
    grid (lbm_partition = partitionForIpus), or N x 1 y slabs."""
    if slabs or n == 1:
        return (n, 1)
    R, C, _ = native.partition(tnx, tny, n)
    return (R, C)


def settle_steps(per_step_s: float, spl: int, budget_s: float = 0.3) -> int:
    """Untimed steps worth ~budget_s of device time (whole launches)."""
    n = int(budget_s / max(per_step_s, 1e-7)) + 1
    n = (n + spl - 1) // spl * spl
    return max(spl, min(n, 20000))


def log(msg: str) -> None:
    print(msg, file=sys.stderr, flush=True)


def measure_copy_gbs(nbytes: int, local_rank: int, reps: int = 5) -> dict:
    """Context for the roofline: a device-to-device copy of one
    lattice's bytes on this GPU, now (torch copy_: read + write = 2 x nbytes
    per copy), best of `reps` after one warm-up.  Never the peak the fractions
    use -- that stays the 8 TB/s HBM figure."""
    import torch
    dev = torch.device("cuda", local_rank)
    n = nbytes // 4
    src = torch.ones(n, dtype=torch.float32, device=dev)
    dst = torch.empty_like(src)
    dst.copy_(src)
    best = float("inf")
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        dst.copy_(src)
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) * 1e-3)
    del src, dst
    torch.cuda.empty_cache()
    gbs = 2 * n * 4 / best / 1e9
    return {"gbs": round(gbs, 1), "bytes": 2 * n * 4, "how": "torch copy_ of one lattice (read + write), best of "
            f"{reps}, live on this box"}


def load_traffic(workload_key: str) -> dict:
    """The committed PMC profile of this workload + kernel (tools/pmc_traffic.py):
    per-launch HBM bytes (gfx950-corrected) and, from the SQ pass, the VALU
    instructions per launch and the VALU pipe's busy fraction; {} if none."""
    f = ROOT / "profiles" / "traffic.json"
    if not f.exists():
        return {}
    try:
        return json.loads(f.read_text()).get(workload_key, {})
    except (ValueError, OSError):
        return {}


def cpu_baseline() -> dict | None:
    """north_star's CPU baseline: main/LbmCpu.cpp as committed (oracle/_ref/lbm_cpu,
    cost only), 128x128 reference problem, all 40 000 steps, one thread."""
    from oracle import oracle  # baseline only
    gold = ROOT / "tests" / "golden" / "params"
    if not oracle.REF_LBMCPU.exists():
        return None
    with tempfile.TemporaryDirectory() as wd:
        r = oracle.run_lbm_cpu(str(gold / "input_128x128.params"), str(gold / "obstacles_128x128.dat"), wd)
    secs = r["compute_s"]
    return {"value": round(128 * 128 * 40000 / secs / 1e6, 2),
            "unit": "MLUPS", "cores": 1, "kind": "reference", "cpu_model": oracle.cpu_model(),
            "sample": f"main/LbmCpu.cpp as committed (-O3, built from the reference source; cost only -- its live "
                      f"kernel fails check.py upstream, SURVEY.md 8c), 128x128 reference problem, all 40000 steps, "
                      f"its own 'Total compute time' {secs:.2f} s (includes its full-lattice printf), 1 thread of "
                      f"{oracle.cpu_model()}"}


def cpu_config1() -> dict | None:
    """BASELINE config 1 plumbing: the reference's LastChance.cpp (correct CPU path)
    on the full 128x128 reference problem, gated by check.py against check/*.dat."""
    from oracle import oracle  # baseline only
    from lbm_amd import check as lcheck
    gold = ROOT / "tests" / "golden"
    if not oracle.REF_LASTCHANCE.exists():
        return None
    with tempfile.TemporaryDirectory() as wd:
        r = oracle.run_reference(str(gold / "params" / "input_128x128.params"),
                                 str(gold / "params" / "obstacles_128x128.dat"), wd)
        res = lcheck.compare(gold / "check" / "128x128.av_vels.dat.gz", gold / "check" / "128x128.final_state.dat.gz",
                             r["av_vels"], r["final_state"])
    secs = r["elapsed_s"]
    return {"program": "main/LastChance.cpp (reference, compiled -O3 -ffp-contract=off)", "grid": "128x128",
            "steps": 40000, "seconds": round(secs, 3), "mlups": round(128 * 128 * 40000 / secs / 1e6, 2),
            "cores": 1, "check_py": "PASS" if res["passed"] else "FAIL",
            "max_av_vels_pct": round(abs(res["av"]["max_diff_pcnt"]), 4) if "av" in res else None,
            "max_final_state_pct": round(abs(res["fs"]["max_diff_pcnt"]), 4) if "fs" in res else None,
            "reynolds": r.get("reynolds")}


def cpu_lastchance_1024() -> dict | None:
    """The reference's own LastChance on a bounded sample of the 1024x1024
    reference problem, single thread on this host."""
    from oracle import oracle  # baseline only
    iters = 500
    gold = ROOT / "tests" / "golden" / "params"
    if not oracle.REF_LASTCHANCE.exists():
        return None
    with tempfile.TemporaryDirectory() as wd:
        pf = Path(wd) / "bench.params"
        pf.write_text(f"1024\n1024\n{iters}\n10\n0.1\n0.01\n1.85\n")
        r = oracle.run_reference(str(pf), str(gold / "obstacles_1024x1024.dat"), wd)
    secs = r["elapsed_s"]
    return {"value": round(1024 * 1024 * iters / secs / 1e6, 2), "unit": "MLUPS", "cores": 1, "kind": "reference",
            "sample": f"main/LastChance.cpp on the 1024x1024 reference problem, first {iters} of 20000 steps, "
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
        e_cells, av = e.store()
        e.run()                      # timed re-run (device events), as LbmRunner's readTimer runs
        secs = e.last_run_seconds()
        used = e.kernel_in_use()
        numerics = e.numerics()
    cells = p.nx * p.ny
    note = ("lattice held on chip (LDS) for the whole run by the resident kernel: bound by the per-step "
            "neighbour hand-off and the collision, not by HBM" if used == "resident" else
            "lattice pair (151 MB) fits the 256 MB Infinity Cache: not an HBM-roofline number")
    return {"grid": "1024x1024", "steps": p.max_iters, "kernel": used, "numerics": numerics,
            "mlups": round(cells * p.max_iters / secs / 1e6, 1),
            "ms_per_step": round(secs / p.max_iters * 1e3, 5),
            "reynolds": lio.reynolds_number(p, float(av[-1])),
            "check_gate": check_gate_1024(p, obst, e_cells, av), "note": note}


def check_gate_1024(p, obst, cells, av) -> dict:
    """The reference's two-file gate (check/check.py:62-147, lbm_amd/check.py
    compare) on the first run's results, in memory: av_vels against the
    reference's check/1024x1024.av_vels.dat, final-state pressure against the
    committed full-run fixture (tests/golden/oracle/1024x1024.final_state_
    pressure.npy.gz, data written by make_golden.py; the reference ships no
    1024^2 final_state).  Also the largest |pressure| difference, 0 in bitwise
    mode."""
    import gzip
    import io as _io
    from lbm_amd import check as lcheck
    gold = ROOT / "tests" / "golden"
    ref_pr = np.load(_io.BytesIO(gzip.decompress(
        (gold / "oracle" / "1024x1024.final_state_pressure.npy.gz").read_bytes())))
    _, _, _, pr = lio.macroscopic(p, obst, cells)
    ny, nx = pr.shape
    coords = np.stack([np.tile(np.arange(nx), ny), np.repeat(np.arange(ny), nx)], 1).astype(np.float64)
    # the written files carry %.12e text: compare the values the text round trip would give
    sim_fs = np.column_stack([coords, np.asarray(pr, np.float64).ravel()])
    ref_fs = np.column_stack([coords, np.asarray(ref_pr, np.float64).ravel()])
    ref_av = lcheck.load_av_vels(gold / "check" / "1024x1024.av_vels.dat.gz")
    sim_av = np.asarray(av, np.float32).astype(np.float64)
    res = lcheck.compare(ref_av, ref_fs, sim_av, sim_fs, 1.0)
    out = {"passed": bool(res["passed"]), "tolerance_pct": 1.0,
           "pressure_max_abs_diff_vs_oracle": float(np.max(np.abs(pr.astype(np.float64) - ref_pr)))}
    if "av" in res:
        out["av_max_diff_pct"] = float(f"{res['av']['max_diff_pcnt']:.3g}")
        out["final_state_max_diff_pct"] = float(f"{res['fs']['max_diff_pcnt']:.3g}")
    else:
        out["reason"] = res["reason"]
    return out


def aux_strong_16384(steps: int, rank: int, world: int, local_rank: int, dist_on: bool, slabs: bool = False,
                     flags: int = 0) -> dict:
    """BASELINE config 4: the fixed 16384x16384 grid (synthetic obstacles) over all
    ranks, RCCL halos overlapped with the interior -- whole-job MLUPS (strong
    scaling; the target is >= 6x at 8 GPUs over 1).  Decomposition: the
    reference's partitionForIpus rule (1x2, 2x2, 2x4: lbm_partition, the
    engine's default), or N x 1 y slabs (slabs=True).  Untimed settle steps
    (>= 0.2 s of device time, same count on every rank) precede the timed
    steps."""
    import torch.distributed as dist
    n = 16384
    p = lio.Params(n, n, steps, 10, 0.1, 0.005, 1.85)
    obst = synthetic_obstacles(n, n)
    numerics = "tolerance" if flags & native.FLAG_TOLERANCE else "bitwise"
    cal = next((v for (_, _, nm), v in _LAUNCH_CAL.items() if nm == numerics), None)
    kw = dict(devices=[local_rank], flags=flags, steps_per_launch=pick_spl(steps, 0, numerics, table=cal))
    if dist_on:
        box = [native.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        kw.update(parts=world, transport=native.TRANSPORT_RCCL, rank=rank, world=world, unique_id=box[0])
        if slabs:
            kw.update(grid=(world, 1))
    g = _RankGate("aux config4", dist_on)

    def setup():
        g.engine = native.Engine(p, obst, **kw)
        g.engine.init_equilibrium()
        g.engine.run_steps(8, accelerate_first=True)
        return g.engine.last_run_seconds() / 8

    per = g.run(setup)
    g.gate("engine setup")
    e = g.engine
    try:
        nset = _agree_max(settle_steps(per, e.steps_per_launch(), 0.2), dist_on)
        g.run(lambda: e.run_steps(nset))
        g.gate("settle steps")
        if dist_on:
            dist.barrier()
        t0 = time.perf_counter()
        g.run(lambda: e.run_steps(steps))
        g.gate("timed steps")   # the all_reduce doubles as the closing barrier
        secs = time.perf_counter() - t0
        kernel_used = e.kernel_in_use()
        spl = e.steps_per_launch()
        rect = e.local_rects()[0]
        av = g.run(lambda: e.store(cells=False, n_av=steps)[1])
        g.gate("store")
    finally:
        e.close()
    finite = _agree_max(0 if np.isfinite(av).all() else 1, dist_on) == 0
    if dist_on:
        import torch
        t = torch.tensor([secs], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        secs = float(t[0])
    R, C, _ = native.partition(n, n, world, *((world, 1) if slabs else (0, 0)))
    return {"grid": f"{n}x{n}", "steps": steps, "settle_steps": nset,
            "decomposition": f"{R}x{C}" + (" (y slabs)" if slabs else " (reference partitionForIpus rule)"),
            "sub_domain": f"{rect[2]}x{rect[3]}", "kernel": kernel_used, "numerics": numerics,
            "launches": launch_plan(steps, spl, kernel_used == "stream"), "av_vels_finite": finite,
            # no rate for a run whose av_vels went non-finite (a broken lattice is not a measurement)
            "mlups": round(n * n * steps / secs / 1e6, 1) if finite else None,
            "ms_per_step": round(secs / steps * 1e3, 4)}


class _RankGate:
    """Host-side phases of a multi-rank aux measurement.  Each phase runs under
    try/except on every rank; gate() then tells every rank, with one
    all_reduce, whether all ranks finished the phase.  An exception on one rank
    so ends the measurement on every rank at the same collective (and closes
    the engine) instead of leaving the others blocked in the next collective
    until the watchdog fires."""

    def __init__(self, what: str, dist_on: bool):
        self.what, self.dist_on, self.err, self.engine = what, dist_on, None, None

    def run(self, fn):
        if self.err is None:
            try:
                return fn()
            except Exception as exc:  # recorded; gate() raises it on every rank
                self.err = exc
        return None

    def gate(self, stage: str) -> None:
        if _agree_max(1 if self.err is not None else 0, self.dist_on):
            if self.engine is not None:
                self.engine.close()
            raise RuntimeError(f"{self.what}: {stage} failed on "
                               + (f"this rank: {type(self.err).__name__}: {self.err}" if self.err else "another rank"))


def _agree_max(v: int, dist_on: bool) -> int:
    """The largest of every rank's value (so all ranks run the same step counts)."""
    if not dist_on:
        return v
    import torch
    import torch.distributed as dist
    t = torch.tensor([v], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return int(t[0])


# D3Q19 aux steps: whole three-step passes (60 = 20 passes, ~0.15 s at 512^3)
D3Q19_STEPS = 60


def aux_d3q19(n: int, steps: int, rank: int, world: int, local_rank: int, dist_on: bool, flags: int = 0) -> dict:
    """BASELINE config 5: D3Q19 n^3 channel (body force between wall planes y = 0 and
    y = n-1), z slabs over all ranks (the engine's default three-step passes:
    RCCL sends three ghost planes each way per pass, overlapped with the slab
    interior), whole-job MLUPS (strong
    scaling: the global grid is fixed).  Untimed settle steps (>= 0.2 s of
    device time) precede the timed steps.  No reference counterpart: parity
    pinned only by the CPU restatement (tests/test_d3q19.py)."""
    import torch.distributed as dist
    p = lio.Params3D(n, n, n, steps, 0.1, 0.001, 1.85)
    obst = lio.channel_obstacles3d(n, n, n)
    kw = dict(devices=[local_rank], flags=flags)
    if dist_on:
        box = [native.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        kw.update(transport=native.TRANSPORT_RCCL, rank=rank, world=world, unique_id=box[0])
    g = _RankGate("aux config5 (D3Q19)", dist_on)

    def setup():
        g.engine = native.Engine3D(p, obst, **kw)
        g.engine.init_equilibrium()
        g.engine.run_steps(4)
        return g.engine.last_run_seconds() / 4

    per = g.run(setup)
    g.gate("engine setup")
    e = g.engine
    try:
        nset = _agree_max(settle_steps(per, 2, 0.2), dist_on)
        g.run(lambda: e.run_steps(nset))
        g.gate("settle steps")
        if dist_on:
            dist.barrier()
        t0 = time.perf_counter()
        g.run(lambda: e.run_steps(steps))
        g.gate("timed steps")   # the all_reduce doubles as the closing barrier
        secs = time.perf_counter() - t0
        dev = e.last_run_seconds()
        nzs = e.local_slabs()[0][1]
        av = g.run(lambda: e.store(cells=False, n_av=steps)[1])
        g.gate("store")
    finally:
        e.close()
    finite = _agree_max(0 if np.isfinite(av).all() else 1, dist_on) == 0
    if dist_on:
        import torch
        t = torch.tensor([secs, dev], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        secs, dev = float(t[0]), float(t[1])
    cells = n ** 3
    # three steps per pass on one slab or z slabs of >= 6 planes, both numerics
    # (step3d_three: 58 x 6 owned of 64 x 12 loaded cells per plane ->
    # (19 x 4 B x (768/348 + 1)) / 3 = 81.2 B per update), the rest in two-step
    # passes (step3d_two: 60 x 8 owned -> (19 x 4 B x (768/480 + 1)) / 2 =
    # 98.8 B) on z slabs of >= 4 planes; 152 B per update for the one-step kernel
    two = nzs >= 4
    three = two and (nzs >= 6 or not dist_on)
    b2, b3 = 19 * 4 * (768 / 480 + 1) / 2, 19 * 4 * (768 / 348 + 1) / 3
    n3 = steps // 3 * 3 if three else 0
    n2 = (steps - n3) // 2 * 2 if two else 0
    alg_b = (n3 * b3 + n2 * b2 + (steps - n3 - n2) * 152) / max(steps, 1)
    # compulsory bytes: each pass moves the lattice through HBM once, 152 B
    # per cell per pass -- 152 / S per update for S steps per pass, without
    # the blocks' overlap re-reads (which b2 / b3 count as algorithmic)
    comp_b = (n3 * 152 / 3 + n2 * 152 / 2 + (steps - n3 - n2) * 152) / max(steps, 1)
    per_gpu_gbs = alg_b * cells / world * steps / dev / 1e9
    comp_gbs = comp_b * cells / world * steps / dev / 1e9
    res = {"grid": f"{n}^3", "steps": steps, "settle_steps": nset, "decomposition": f"{world} z slabs",
            "numerics": "tolerance" if flags & native.FLAG_TOLERANCE else "bitwise",
            "kernel": (f"step3d_three ({n3 // 3} passes of 3 steps) + step3d_two ({n2 // 2} of 2)" if three else
                       "step3d_two (2 steps per pass)" if two else "step3d_pair (1 step per launch)"),
            "av_vels_finite": finite, "mlups": round(cells * steps / secs / 1e6, 1) if finite else None,
            "ms_per_step": round(secs / steps * 1e3, 4),
            "hbm_gbs_per_gpu": round(per_gpu_gbs, 1), "hbm_frac": round(per_gpu_gbs / HBM_PEAK_GBS, 4),
            "compulsory_b_per_update": round(comp_b, 2),
            "hbm_gbs_compulsory_per_gpu": round(comp_gbs, 1),
            "hbm_frac_compulsory": round(comp_gbs / HBM_PEAK_GBS, 4),
            "effective_gbs_per_gpu": round(152 * cells / world * steps / dev / 1e9, 1),
            "note": f"hbm_frac: {alg_b:.1f} B per update including the blocks' overlap re-reads; hbm_frac_compulsory: "
                    f"{comp_b:.1f} B per update, the lattice once per pass (152 B = 19 fp32 loads + stores per cell; "
                    "effective_gbs on that basis per step); parity unpinned upstream (no 3-D reference)"}
    # the committed PMC passes of this pass on one GPU (tools/pmc_traffic.py,
    # profiles/traffic.json): HBM bytes per three-step pass against the
    # compulsory 152 B x cells, the VALU pipe's busy fraction
    prof = load_traffic(f"{n}^3/three{'t' if flags & native.FLAG_TOLERANCE else 'b'}") if world == 1 and three else {}
    if prof:
        res["pmc"] = {"hbm_bytes_per_pass": prof.get("hbm_bytes_per_launch"),
                      "ratio_to_compulsory": prof.get("ratio_to_algorithmic"),
                      "valu_busy": (prof.get("valu") or {}).get("busy_frac"),
                      "correction": prof.get("correction"), "profile": prof.get("profile")}
    return res


def _check_cases(world: int):
    """The multi-rank self-check's cases: (name, global nx, ny, grid (R, C) or (0, 0) for the
    reference rule, numerics, steps, flags, perturbed start)."""
    n = 2048
    # config 4's per-rank shape at a quarter of its height: 16384^2 over N ranks
    # by the reference rule is (16384 / C) x (16384 / R) per rank (4096 x 8192 in
    # 2x4 at N = 8); the check runs (16384 / C) x (4096 / R) per rank (4096 x 2048)
    # on the same R x C grid, with the tolerance collision's driver plan (2 x 10)
    R4, C4, _ = native.partition(16384, 16384, world)
    cases = []
    for mode, steps, flags in (("bitwise", 13, 0), ("tolerance", 27, native.FLAG_TOLERANCE)):
        for name, grid in (("reference_rule", (0, 0)), ("slabs", (world, 1))):
            cases.append((f"{mode}_{name}", n, n, grid, mode, steps, flags, True))
    cases.append(("tolerance_config4_shape", 16384, 4096, (R4, C4), "tolerance", 20, native.FLAG_TOLERANCE, False))
    return cases


def multi_rank_check(rank: int, world: int, local_rank: int) -> dict:
    """N > 1, untimed, before the timed region: the fused stream kernel over all
    ranks (RCCL halos) against a single-domain run of the same library and mode
    on every rank's own GPU (each rank compares its own block bitwise; no
    gather).  Cases (_check_cases): a 2048^2 problem with random obstacles and a
    perturbed start on the reference partitionForIpus blocks and on N x 1 slabs,
    bitwise collision 13 steps (two 6-step launches + a one-step remainder) and
    tolerance collision 27 steps (10 + 10 + a fused 7-step remainder); and
    config 4's per-rank block shape (a quarter of its height: 4096 x 2048 per
    rank in 2x4 at N = 8) in tolerance mode, 20 steps (2 x 10, the driver's
    timed plan).
    tests/test_gpu_parity.py pins the bitwise collision to the CPU oracle; the
    tolerance collision is decomposition-invariant (tests/test_gpu_tolerance.py).
    Every rank runs the same collective sequence whatever happens on it: an
    exception in a case is recorded as that rank's result and the per-case
    all_gather_object still runs.  (A rank that fails inside an RCCL call
    leaves the others waiting; bench's main watchdog ends that, exit 4.)
    Reference: StructuredGridUtils.hpp:498-522 (split), :805-851 (halos)."""
    import torch.distributed as dist
    results = {}
    for name, nx, ny, grid, mode, steps, flags, perturbed in _check_cases(world):
        rng = np.random.default_rng(2024)
        obst = synthetic_obstacles(nx, ny)
        obst[rng.random((ny, nx)) < 0.02] = 1
        p = lio.Params(nx, ny, steps, 10, 0.1, 0.005, 1.85)
        cells0 = (lio.init_cells(p) * (1 + 0.02 * rng.standard_normal((ny, nx, 9)))).astype(np.float32) \
            if perturbed else None
        box = [native.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        mine = {"bitwise": False}
        try:
            R, C, rects = native.partition(nx, ny, world, *grid)
            x0, y0, w, h = (int(v) for v in rects[rank])
            with native.Engine(p, obst, parts=world, grid=grid, transport=native.TRANSPORT_RCCL, rank=rank,
                               world=world, devices=[local_rank], unique_id=box[0], kernel=native.KERNEL_STREAM,
                               flags=flags) as e:
                if perturbed:
                    e.load_cells_local([cells0[y0:y0 + h, x0:x0 + w]])
                else:
                    e.init_equilibrium()
                e.run_steps(steps, accelerate_first=True)
                stats = e.run_stats()
                blocks, av = e.store_local(n_av=steps)
            with native.Engine(p, obst, devices=[local_rank], kernel=native.KERNEL_STREAM, flags=flags) as e1:
                if perturbed:
                    e1.load_cells(cells0)
                else:
                    e1.init_equilibrium()
                e1.run_steps(steps, accelerate_first=True)
                ref, ref_av = e1.store(n_av=steps)
            mine = {"decomposition": f"{R}x{C}", "block": f"{w}x{h}", "steps": steps, "launches": list(stats),
                    "bitwise": bool(np.array_equal(blocks[0], ref[y0:y0 + h, x0:x0 + w])),
                    "finite": bool(np.isfinite(blocks[0]).all() and np.isfinite(av).all()),
                    "av_vels_rel": float(np.max(np.abs(av - ref_av) / np.abs(ref_av)))}
            mine["bitwise"] = mine["bitwise"] and mine["finite"]
        except Exception as exc:  # recorded; the collective sequence continues
            mine = {"bitwise": False, "error": f"{type(exc).__name__}: {exc}"}
        every = [None] * world
        dist.all_gather_object(every, mine)
        bad = [r for r, m in enumerate(every) if not m.get("bitwise")]
        results[name] = dict(every[0], ranks_failed=bad)
        if bad:
            results[name]["bitwise"] = False
            errors = {r: every[r]["error"] for r in bad if every[r].get("error")}
            if errors:
                results[name]["errors"] = errors
    return {"passed": all(not r["ranks_failed"] for r in results.values()), "cases": results}


CHECK_FAILED_EXIT = 5


def gate_multi_rank(mrc: dict, rank: int, n: int, mwd=None) -> None:
    """A failed self-check is fatal before anything is timed: rank 0 prints
    check_failed_line (value null, the cases) and every rank exits with
    CHECK_FAILED_EXIT (5).  Every rank already holds the same per-case verdict
    (all_gather_object); an exception outside the cases is local to one rank,
    so the ranks agree on the outcome explicitly first."""
    ok = _agree_max(0 if mrc.get("passed") else 1, True) == 0
    if ok:
        return
    if rank == 0:
        print(json.dumps(check_failed_line(mrc, n)), flush=True)
    log(f"multi-rank self-check failed; exiting with status {CHECK_FAILED_EXIT} before the timed region")
    if mwd is not None:
        mwd.cancel()
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(CHECK_FAILED_EXIT)


def check_failed_line(mrc: dict, n: int) -> dict:
    """The line printed (rank 0) when the multi-rank self-check fails: no value."""
    return {"metric": METRIC, "value": None, "unit": "MLUPS", "n_gpus": n, "higher_is_better": True,
            "error": "multi-rank self-check failed: the decomposed run differs from the single-domain run "
                     "(or raised); nothing was timed",
            "multi_rank_bitwise": False, "multi_rank_check": mrc}


# Fallback only (calibrate_launch_ms measures these on the box at bench start):
# device ms per fused launch of S steps at 8192^2 (profiles/r03/ab_spl_ow16.log,
# 16-column aligned strips; tolerance S >= 7: the round-4 LP form with one row
# per iteration, profiles/r04/ab_lp10.log): bitwise and tolerance collision; a
# launch of 2..5 steps is bound by the lattice pass (~1.1 ms); a one-step
# (vec4) launch 0.81 ms.
LAUNCH_MS = {"bitwise": {2: 1.12, 3: 1.07, 4: 1.10, 5: 1.18, 6: 1.39},
             "tolerance": {2: 1.11, 3: 1.07, 4: 1.08, 5: 1.10, 6: 1.10, 7: 1.21, 8: 1.33, 9: 1.50, 10: 1.55}}
ONE_STEP_MS = 0.81
_LAUNCH_CAL: dict = {}
BOUND_FRAC = 0.75   # a roofline fraction at or above this names the bound


def _agree_max_f(v: float, dist_on: bool) -> float:
    """The largest of every rank's float value."""
    if not dist_on:
        return v
    import torch
    import torch.distributed as dist
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0])


def calibrate_launch_ms(tnx: int, tny: int, numerics: str, local_rank: int, dist_on: bool, reps: int = 4) -> dict:
    """Device ms per fused launch of S steps, for every S the collision allows
    (bitwise 2..6, tolerance 2..10), and per one-step launch, measured on THIS
    GPU at the bench tile with the library's own events (a single-domain
    stream engine per S, placement probe included as in the timed engine),
    max over ranks so every rank picks the same S.  Untimed, before the
    warm-up; cached per tile and numerics.  Replaces reading LAUNCH_MS, which
    a kernel change would silently invalidate (LAUNCH_MS stays the fallback
    when a calibration engine cannot be built)."""
    key = (tnx, tny, numerics)
    if key in _LAUNCH_CAL:
        return _LAUNCH_CAL[key]
    smax = 10 if numerics == "tolerance" else 6
    flags = native.FLAG_TOLERANCE if numerics == "tolerance" else 0
    p = lio.Params(tnx, tny, 1, 10, 0.1, 0.005, 1.85)
    obst = synthetic_obstacles(tnx, tny)
    ms, one = {}, None
    t0 = time.perf_counter()
    try:
        for i, S in enumerate(range(smax, 1, -1)):
            with native.Engine(p, obst, devices=[local_rank], kernel=native.KERNEL_STREAM, flags=flags,
                               steps_per_launch=S) as e:
                e.init_equilibrium()
                e.run_steps((60 if i == 0 else 2) * S, accelerate_first=True)   # clock ramp, then warm
                e.run_steps(reps * S)
                if e.run_stats() != (reps, 0):
                    raise RuntimeError(f"S = {S}: launches {e.run_stats()}, expected ({reps}, 0)")
                ms[S] = e.last_run_seconds() / reps * 1e3
        # the one-step launch a K mod S = 1 remainder runs (vec4 at these widths)
        with native.Engine(p, obst, devices=[local_rank], kernel=native.KERNEL_VEC4,
                           flags=native.FLAG_ONE_STEP) as e:
            e.init_equilibrium()
            e.run_steps(2, accelerate_first=True)
            e.run_steps(reps)
            if e.run_stats() != (0, reps):
                raise RuntimeError(f"one-step: launches {e.run_stats()}, expected (0, {reps})")
            one = e.last_run_seconds() / reps * 1e3
    except Exception as exc:  # recorded; the fallback table is used
        log(f"launch calibration failed ({type(exc).__name__}: {exc}); using LAUNCH_MS")
        ms, one = None, None
    if _agree_max(1 if ms is None else 0, dist_on):   # any rank failed: every rank uses the fallback
        res = {"source": "LAUNCH_MS fallback (profiles/r04)", "ms": dict(LAUNCH_MS[numerics]), "one_step_ms": ONE_STEP_MS}
    else:
        res = {"source": f"measured at bench start on this GPU ({tnx}x{tny}, {reps} launches per S, "
                         f"{time.perf_counter() - t0:.1f} s)",
               "ms": {S: round(_agree_max_f(v, dist_on), 4) for S, v in sorted(ms.items())},
               "one_step_ms": round(_agree_max_f(one, dist_on), 4)}
    _LAUNCH_CAL[key] = res
    return res


def pick_spl(steps: int, requested: int, numerics: str = "bitwise", fused_remainder: bool = True,
             table: dict | None = None) -> int:
    """Steps per fused launch for a timed run of `steps` steps: the caller's
    choice if given, else the S whose launches finish `steps` soonest, counting
    the remainder steps % S as the library runs it (include/lbm_hip.h: one
    fused launch when >= 2 steps, else one one-step launch).  `table`: a
    calibrate_launch_ms result (else the LAUNCH_MS fallback) -- with it,
    bitwise: the driver's 20-step run is four 5-step launches, 1000 steps 166
    six-step launches + a 4-step one; tolerance: 2 x 10 and 100 x 10."""
    if requested:
        return requested
    ms = {int(k): v for k, v in table["ms"].items()} if table else LAUNCH_MS[numerics]
    one = table["one_step_ms"] if table else ONE_STEP_MS

    def est(S):
        r = steps % S
        tail = ms[r] if (r >= 2 and fused_remainder) else r * one
        return (steps // S) * ms[S] + tail

    return min(sorted(ms, reverse=True), key=est) if steps > 0 else max(ms)


def measure_weak(tnx: int, tny: int, R: int, C: int, args, kernel: int, kflags: int, rank: int, world: int,
                 local_rank: int, dist_on: bool) -> dict:
    """K timed steps of the weak-scaling workload: R x C tiles of tnx x tny cells,
    one per rank (R*C == world), after W warm-up and the settle steps."""
    import torch
    import torch.distributed as dist
    nx, ny = tnx * C, tny * R
    p = lio.Params(nx, ny, args.steps, 10, 0.1, 0.005, 1.85)
    obst = synthetic_obstacles(nx, ny)
    uid = None
    if dist_on:
        box = [native.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        uid = box[0]
    numerics = "tolerance" if kflags & native.FLAG_TOLERANCE else "bitwise"
    cal = None
    if kernel in (native.KERNEL_AUTO, native.KERNEL_STREAM) and not args.spl:
        cal = calibrate_launch_ms(tnx, tny, numerics, local_rank, dist_on) if args.calibrate else None
        spl = pick_spl(args.steps, 0, numerics, table=cal)
    else:
        spl = args.spl
    eng = native.Engine(p, obst, parts=world, grid=(R, C),
                        transport=native.TRANSPORT_RCCL if dist_on else native.TRANSPORT_LOCAL,
                        rank=rank, world=world, devices=[local_rank], unique_id=uid, kernel=kernel, flags=kflags,
                        steps_per_launch=spl)
    try:
        eng.init_equilibrium()
        spl = eng.steps_per_launch()
        if args.warmup > 0:
            eng.run_steps(args.warmup, accelerate_first=True)
            per_step = eng.last_run_seconds() / args.warmup
        else:
            eng.run_steps(spl, accelerate_first=True)
            per_step = eng.last_run_seconds() / spl
        nset = _agree_max(settle_steps(per_step, spl, args.settle) if args.settle > 0 else 0, dist_on)
        set_secs = 0.0
        if nset > 0:
            eng.run_steps(nset)
            set_secs = eng.last_run_seconds()

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
        return {"nx": nx, "ny": ny, "elapsed": elapsed, "dev_secs": dev_secs, "finite": bool(np.all(np.isfinite(av))),
                "kernel": eng.kernel_in_use(), "spl": eng.steps_per_launch(), "numerics": eng.numerics(),
                "launches": eng.run_stats(), "calibration": cal,
                "settle": {"steps": nset, "device_s": round(set_secs, 4),
                           "why": "GPU clock ramp over the first ~20-30 ms of back-to-back work "
                                  "(tools/settle_probe.py); untimed, same count on every rank"}}
    finally:
        eng.close()


TOLERANCE_NOTE = ("LBM_FLAG_TOLERANCE (include/lbm_hip.h): IEEE fp32, one reciprocal of rho per cell (v_rcp_f32, 1 "
                  "ulp) and FMA-reassociated BGK terms instead of LastChance.cpp's two correctly rounded "
                  "divisions; stated tolerance (tests/test_gpu_tolerance.py): every population within 2e-5 "
                  "relative of the CPU oracle for runs of up to 100 steps (8192^2, 16384^2) and within 2e-3 over "
                  "the full reference runs on all four reference grids (20000 steps at 1024^2, measured 4.3e-4; "
                  "at most 9.0e-4 on any grid), av_vels within 2e-3 (3e-3 over the full runs, measured <= 1.5e-3), "
                  "the two-file check.py gate (1 %) passes on "
                  "all four grids at full maxIters, and the lattice does not depend on steps per launch or "
                  "decomposition")


def launch_plan(steps: int, spl: int, stream: bool) -> str:
    """The launches a run of `steps` steps makes (include/lbm_hip.h)."""
    q, r = divmod(steps, spl)
    if r >= 2 and stream:
        return f"{q} x {spl} + 1 x {r} (fused remainder)"
    return f"{q} x {spl}" + (f" + {r} x 1" if r else "")


WATCHDOG_EXIT = 3


class AuxWatchdog:
    """Bounds the aux phase.  The main measurement is done when it starts; an aux
    that hangs (e.g. one rank failed an aux and left the others waiting in an
    RCCL exchange) would otherwise keep rank 0 from ever printing the line.  Past
    the budget, rank 0 prints the line with the aux finished so far plus a note,
    and every rank exits with status WATCHDOG_EXIT (3): the launcher and CI see
    that an aux hung, while the printed line still carries `value`."""

    def __init__(self, budget_s: float, out: dict, rank: int):
        self.out, self.rank = out, rank
        self.lock = threading.Lock()
        self.printed = False
        self.timer = None
        if budget_s > 0:
            self.timer = threading.Timer(budget_s, self._fire, args=(budget_s,))
            self.timer.daemon = True
            self.timer.start()

    def _print(self, out: dict) -> None:
        with self.lock:
            if self.printed:
                return
            self.printed = True
            if self.rank == 0:
                print(json.dumps(out), flush=True)

    def _fire(self, budget_s: float) -> None:
        try:
            out = json.loads(json.dumps(self.out))  # a consistent copy
        except (TypeError, ValueError, RuntimeError):
            out = {k: v for k, v in self.out.items() if k != "aux"}
        out.setdefault("aux", {})["watchdog"] = f"aux phase exceeded {budget_s:.0f} s; the remaining aux were skipped"
        self._print(out)
        log(f"aux watchdog: {budget_s:.0f} s exceeded, exiting with status {WATCHDOG_EXIT}")
        os._exit(WATCHDOG_EXIT)

    def finish(self) -> None:
        if self.timer is not None:
            self.timer.cancel()
        self._print(self.out)


MAIN_WATCHDOG_EXIT = 4


def main_watchdog(budget_s: float, rank: int, n: int) -> threading.Timer | None:
    """N > 1: bounds the multi-rank check and the timed measurement (RCCL
    between real devices runs for the first time on the driver's multi-GPU
    node).  Past the budget rank 0 prints a line that says so and every rank
    exits with MAIN_WATCHDOG_EXIT (4), so a hung exchange frees the node
    instead of holding it until the launcher's limit."""
    if budget_s <= 0 or n <= 1:
        return None

    def fire():
        if rank == 0:
            print(json.dumps({"metric": METRIC, "value": None, "unit": "MLUPS", "n_gpus": n,
                              "error": f"multi-rank check / timed measurement exceeded {budget_s:.0f} s"}), flush=True)
        log(f"main watchdog: {budget_s:.0f} s exceeded, exiting with status {MAIN_WATCHDOG_EXIT}")
        os._exit(MAIN_WATCHDOG_EXIT)

    t = threading.Timer(budget_s, fire)
    t.daemon = True
    t.start()
    return t


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--settle", type=float, default=0.3,
                    help="untimed settle steps worth this many seconds of device time after the warm-up (0: none)")
    ap.add_argument("--tile", default="8192x8192", help="cells per GPU, NXxNY")
    ap.add_argument("--kernel", default="auto", choices=["auto", "resident", "stream", "step2", "vec4", "scalar", "pipeline"],
                    help="stream: fused S-step register-streaming kernel; step2: fused two-step LDS kernel; "
                         "vec4/scalar: one step per launch; auto: the library's choice")
    ap.add_argument("--spl", type=int, default=0,
                    help="stream: time steps per launch (2..6, 2..10 with tolerance numerics; 0 = the fastest for "
                         "--steps by the measured launch times, pick_spl)")
    ap.add_argument("--numerics", default="tolerance", choices=["tolerance", "bitwise"],
                    help="value's collision: tolerance = LBM_FLAG_TOLERANCE (fp32, within the stated tolerance of "
                         "the reference: north_star's 'within a stated fp32 tolerance'); bitwise = every population "
                         "bit-identical to LastChance.cpp; the other mode is measured too (aux)")
    ap.add_argument("--no-calibrate", dest="calibrate", action="store_false",
                    help="pick S from the LAUNCH_MS fallback table instead of timing every S on this GPU first")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-aux", action="store_true")
    ap.add_argument("--no-d3q19", action="store_true")
    ap.add_argument("--no-strong", action="store_true", help="skip the 16384^2 strong-scaling aux (config 4)")
    ap.add_argument("--d3q19-n", type=int, default=512, help="D3Q19 aux grid edge (BASELINE config 5: 512)")
    ap.add_argument("--main-budget", type=float, default=600.0,
                    help="N > 1: seconds the multi-rank check plus the timed measurement may take (0: no limit)")
    ap.add_argument("--aux-budget", type=float, default=300.0,
                    help="seconds the aux measurements may take after the main one; past it rank 0 prints the "
                         "line with the aux done so far and every rank exits (0: no limit)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    n = world
    kernel = {"auto": native.KERNEL_AUTO, "resident": native.KERNEL_RESIDENT, "pipeline": native.KERNEL_PIPELINE,
              "stream": native.KERNEL_STREAM, "step2": native.KERNEL_STEP2,
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
    R, C = weak_grid(n, tnx, tny)
    mwd = main_watchdog(args.main_budget, rank, n)
    mrc = None
    if dist_on:
        try:
            mrc = multi_rank_check(rank, world, local_rank)
        except Exception as exc:  # recorded, never silently dropped
            mrc = {"passed": False, "error": f"{type(exc).__name__}: {exc}"}
        log(f"multi-rank bitwise check: {mrc}")
        gate_multi_rank(mrc, rank, n, mwd)
    tol_main = args.numerics == "tolerance" and args.kernel in ("auto", "stream")
    kflags_main = kflags | (native.FLAG_TOLERANCE if tol_main else 0)
    m = measure_weak(tnx, tny, R, C, args, kernel, kflags_main, rank, world, local_rank, dist_on)
    nx, ny, elapsed, dev_secs = m["nx"], m["ny"], m["elapsed"], m["dev_secs"]
    kernel_used, steps_per_launch = m["kernel"], m["spl"]
    if mwd is not None:
        mwd.cancel()

    total_cells = nx * ny
    value = total_cells * args.steps / elapsed / 1e6
    # every launch (fused S steps, a fused remainder, or one step) moves the
    # lattice through HBM once: 72 algorithmic bytes per cell per launch
    launches = max(m["launches"][0] + m["launches"][1], 1)
    per_launch_s = dev_secs / launches
    cells_per_gpu = tnx * tny
    achieved = BYTES_PER_UPDATE * cells_per_gpu / per_launch_s / 1e9
    effective = BYTES_PER_UPDATE * cells_per_gpu * args.steps / dev_secs / 1e9
    wl_key = (f"{tnx}x{tny}/{kernel_used}" + (str(steps_per_launch) if kernel_used == "stream" else "") +
              ("t" if m["numerics"] == "tolerance" else ""))
    prof = load_traffic(wl_key)
    traffic = prof.get("hbm_bytes_per_launch")
    valu = prof.get("valu") or {}
    # Which bound binds, from three fractions of one
    # launch: the per-pass algorithmic bytes / launch time / HBM peak (frac),
    # the PMC-counted HBM bytes / launch time / peak (what the channels really
    # moved), and the VALU pipe's busy share of the SIMD cycles in quad-cycle
    # units (4 x SQ_ACTIVE_INST_VALU / (SIMDs x GRBM_GUI_ACTIVE / 8),
    # tools/pmc_traffic.py).  A bound is named only when its fraction reaches
    # BOUND_FRAC; when none does, the launch is latency-bound (waits on loads,
    # LDS and dependency chains), and it is called that.
    frac_pass = achieved / HBM_PEAK_GBS
    frac_counter = (traffic / per_launch_s / 1e9 / HBM_PEAK_GBS) if traffic else None
    frac_valu = valu.get("busy_frac")
    fracs = {"hbm": max(frac_pass, frac_counter or 0.0), "valu": frac_valu or 0.0}
    top = max(fracs, key=fracs.get)
    bound = top if fracs[top] >= BOUND_FRAC else "latency"
    try:
        copy = measure_copy_gbs(BYTES_PER_UPDATE // 2 * cells_per_gpu, local_rank)
        copy["pass_vs_copy"] = round(achieved / copy["gbs"], 4)
    except Exception as exc:  # context only: recorded, never fatal
        copy = {"error": f"{type(exc).__name__}: {exc}"}

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
                   "parallelism": (f"{R}x{C} blocks (reference partitionForIpus rule), one per GPU, RCCL halo "
                                   f"exchange overlapped with the interior" if n > 1 else "single GPU"),
                   "kernel": kernel_used},
        "settle": m["settle"],
        "roofline": {"bound": bound, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "frac_counter_bytes": round(frac_counter, 4) if frac_counter is not None else None,
                     "frac_valu_issue": frac_valu,
                     "bound_rule": (f"the largest of frac / frac_counter_bytes (HBM) and frac_valu_issue (VALU) "
                                    f"if >= {BOUND_FRAC}, else 'latency'"),
                     "bytes_per_launch": BYTES_PER_UPDATE * cells_per_gpu,
                     "cell_updates_per_launch": steps_per_launch * cells_per_gpu,
                     "steps_per_launch": steps_per_launch,
                     "avg_launch_ms": round(per_launch_s * 1e3, 5),
                     # SURVEY 8(d) form: 72 B x cell updates / s; a fused S-step launch moves
                     # the lattice through HBM once per S updates, so this can exceed the peak
                     "effective_gbs": round(effective, 1),
                     "effective_frac": round(effective / HBM_PEAK_GBS, 4),
                     # VALU instructions per launch and the pipe's busy fraction, same profile
                     "valu": prof.get("valu") or None, "profile": prof.get("profile"),
                     # what a plain device copy of the same bytes reaches on this box, now
                     "device_copy": copy},
        "av_vels_finite": m["finite"],
        "numerics": m["numerics"],
        "launches": {"fused": m["launches"][0], "one_step": m["launches"][1],
                     "plan": launch_plan(args.steps, steps_per_launch, kernel_used == "stream"),
                     "calibration": m["calibration"]},
    }
    if m["numerics"] == "tolerance":
        out["tolerance"] = TOLERANCE_NOTE
    if mrc is not None:
        out["multi_rank_bitwise"] = bool(mrc.get("passed"))
        out["multi_rank_check"] = mrc
    aux = out.setdefault("aux", {})
    watchdog = AuxWatchdog(args.aux_budget, out, rank)
    if not args.no_aux and args.kernel in ("auto", "stream") and kernel_used == "stream":
        # the same workload and step count with the other collision: bitwise
        # (LastChance.cpp arithmetic) when `value` is the tolerance mode, and
        # vice versa (LBM_FLAG_TOLERANCE, include/lbm_hip.h)
        other = "bitwise" if m["numerics"] == "tolerance" else "tolerance"
        try:
            mt = measure_weak(tnx, tny, R, C, args, kernel, kflags | (native.FLAG_TOLERANCE if other == "tolerance"
                                                                     else 0), rank, world, local_rank, dist_on)
            lt = mt["dev_secs"] / max(mt["launches"][0] + mt["launches"][1], 1)
            aux[f"stream{mt['spl']}_{other}"] = {
                "mlups": round(mt["nx"] * mt["ny"] * args.steps / mt["elapsed"] / 1e6, 1),
                "ms_per_step": round(mt["elapsed"] / args.steps * 1e3, 5), "numerics": mt["numerics"],
                "steps_per_launch": mt["spl"], "launches": launch_plan(args.steps, mt["spl"], True),
                "avg_launch_ms": round(lt * 1e3, 5),
                "hbm_frac_per_pass": round(BYTES_PER_UPDATE * tnx * tny / lt / 1e9 / HBM_PEAK_GBS, 4),
                **({"tolerance": TOLERANCE_NOTE} if other == "tolerance" else
                   {"parity": "every population bit-identical to the CPU oracle (LastChance.cpp:226-262 restated), "
                              "tests/test_gpu_parity.py"})}
        except Exception as exc:
            aux[f"stream_{other}"] = {"error": str(exc)}
    if n > 1 and not args.no_aux:
        try:
            ms = measure_weak(tnx, tny, n, 1, args, kernel, kflags_main, rank, world, local_rank, dist_on)
            aux["weak_slabs"] = {"decomposition": f"{n}x1 (y slabs)", "global_grid": f"{ms['nx']}x{ms['ny']}",
                                 "mlups": round(ms["nx"] * ms["ny"] * args.steps / ms["elapsed"] / 1e6, 1),
                                 "ms_per_step": round(ms["elapsed"] / args.steps * 1e3, 5), "kernel": ms["kernel"]}
        except Exception as exc:
            aux["weak_slabs"] = {"error": str(exc)}
    if not args.no_aux and not args.no_strong:
        for key, slabs in (("config4_16384x16384", False), ("config4_slabs", True)):
            if slabs and n == 1:
                continue
            try:
                aux[key] = aux_strong_16384(100, rank, world, local_rank, dist_on, slabs=slabs,
                                            flags=kflags_main & native.FLAG_TOLERANCE)
            except Exception as exc:
                aux[key] = {"error": str(exc)}
    if not args.no_aux and not args.no_d3q19:
        try:
            aux["config5_d3q19"] = aux_d3q19(args.d3q19_n, D3Q19_STEPS, rank, world, local_rank, dist_on)
        except Exception as exc:
            aux["config5_d3q19"] = {"error": str(exc)}
        try:
            aux["config5_d3q19_tolerance"] = aux_d3q19(args.d3q19_n, D3Q19_STEPS, rank, world, local_rank, dist_on,
                                                       flags=native.FLAG_TOLERANCE)
        except Exception as exc:
            aux["config5_d3q19_tolerance"] = {"error": str(exc)}
    if rank == 0 and n == 1:
        if not args.no_aux:
            try:
                aux["config2_1024x1024"] = aux_1024(kernel, kflags, args.spl)
            except Exception as exc:
                aux["config2_1024x1024"] = {"error": str(exc)}
            try:  # the same problem with LBM_FLAG_TOLERANCE (packed resident tiles, reciprocal collision)
                aux["config2_1024x1024_tolerance"] = aux_1024(kernel, kflags | native.FLAG_TOLERANCE, args.spl)
            except Exception as exc:
                aux["config2_1024x1024_tolerance"] = {"error": str(exc)}
        if not args.no_cpu_baseline:
            for key, fn in (("cpu_baseline", cpu_baseline), ("cpu_config1_128x128", cpu_config1),
                            ("cpu_lastchance_1024x1024", cpu_lastchance_1024),
                            ("cpu_baseline_threads", cpu_baseline_threads)):
                try:
                    r = fn()
                except Exception as exc:
                    r = None
                    log(f"{key} failed: {exc}")
                if key == "cpu_baseline":
                    out["cpu_baseline"] = r if r is not None else cpu_lastchance_1024()
                elif r is not None:
                    aux[key] = r
    if not aux:
        out.pop("aux")
    watchdog.finish()
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
