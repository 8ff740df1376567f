"""bench.py's multi-rank self-check at N > 1 (CPU, gloo world of 2): the check
must keep every rank in the same collective sequence whatever fails on one of
them, and a failed check is fatal before anything is timed -- rank 0 prints a
line with "value": null and the per-case results, and every rank exits with
bench.CHECK_FAILED_EXIT (5).

The engines are replaced by a stand-in whose "lattice" is the initial state
(so decomposed and single-domain runs agree unless a failure is injected):
what is under test is bench's control flow around them (multi_rank_check,
gate_multi_rank), not the kernels (tests/test_multigpu.py runs those on
>= 2 GPUs, tests/test_gpu_parity.py on one).
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import PKG, ROOT

WORKER = r'''
import json, os, sys
sys.path[:0] = [{root!r}, {pkg!r}]
import numpy as np
import torch.distributed as dist
import bench

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
inject = os.environ.get("INJECT", "")
dist.init_process_group("gloo", rank=rank, world_size=world)


class FakeEngine:
    case = None

    def __init__(self, p, obst, **kw):
        self.p, self.kw = p, kw
        self.decomposed = "parts" in kw
        self.state = None
        if inject == "raise_create_ref_rank0" and rank == 0 and not self.decomposed and FakeEngine.case == "b":
            raise RuntimeError("injected: single-domain engine failed on rank 0")

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

    def _rect(self):
        R, C, rects = bench.native.partition(self.p.nx, self.p.ny, world, *self.kw.get("grid", (0, 0)))
        return rects[rank]

    def load_cells_local(self, blocks):
        self.state = np.array(blocks[0])

    def load_cells(self, cells):
        self.state = np.array(cells)

    def init_equilibrium(self):
        full = bench.lio.init_cells(self.p)
        if self.decomposed:
            x0, y0, w, h = self._rect()
            full = full[y0:y0 + h, x0:x0 + w]
        self.state = np.array(full)

    def run_steps(self, steps, accelerate_first=False):
        if inject == "raise_run_rank1" and rank == 1 and self.decomposed and FakeEngine.case == "b":
            raise RuntimeError("injected: decomposed run failed on rank 1")
        if inject == "corrupt_rank1" and rank == 1 and self.decomposed and FakeEngine.case == "b":
            self.state[0, 0, 0] += 1.0

    def run_stats(self):
        return (1, 0)

    def store_local(self, n_av=1):
        return [self.state], np.ones(n_av, np.float32)

    def store(self, n_av=1):
        return self.state, np.ones(n_av, np.float32)


def cases(world):
    out = []
    for name, grid, flags, pert in (("a", (0, 0), 0, True), ("b", (world, 1), 4, False), ("c", (1, world), 4, True)):
        out.append((name, 24, 16, grid, "m", 3, flags, pert))
    return out


orig_cases = cases


def tracked_cases(world):
    for c in orig_cases(world):
        FakeEngine.case = c[0]
        yield c


bench.native.Engine = FakeEngine
bench.native.rccl_unique_id = lambda: b"u" * 128
bench._check_cases = tracked_cases
mrc = bench.multi_rank_check(rank, world, 0)
print(json.dumps({{"rank": rank, "mrc": mrc}}), file=sys.stderr, flush=True)
bench.gate_multi_rank(mrc, rank, world)
print("PASSED_GATE", flush=True)
dist.barrier()
dist.destroy_process_group()
'''


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(inject: str, timeout: float = 120, world: int = 2):
    code = WORKER.format(root=str(ROOT), pkg=str(PKG))
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), INJECT=inject, OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    out = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=timeout)
            out.append((p.returncode, o, e))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return out


def _bench_const(name):
    sys.path[:0] = [str(ROOT), str(PKG)]
    import bench
    return getattr(bench, name)


def test_check_passes_and_gate_lets_the_run_continue():
    out = _run("")
    for rc, o, e in out:
        assert rc == 0, e
        assert "PASSED_GATE" in o


@pytest.mark.parametrize("inject,rank_failed", [("corrupt_rank1", 1), ("raise_run_rank1", 1),
                                                ("raise_create_ref_rank0", 0)])
def test_failed_check_is_fatal_on_every_rank(inject, rank_failed):
    exit_code = _bench_const("CHECK_FAILED_EXIT")
    assert exit_code == 5
    out = _run(inject)
    for rc, o, e in out:
        assert rc == exit_code, e
        assert "PASSED_GATE" not in o
    lines = [ln for ln in out[0][1].splitlines() if ln.startswith("{")]  # gloo logs to stdout too
    assert len(lines) == 1, out[0][1]
    d = json.loads(lines[0])
    assert d["value"] is None and d["n_gpus"] == 2 and d["multi_rank_bitwise"] is False
    cases = d["multi_rank_check"]["cases"]
    assert cases["a"]["ranks_failed"] == [] and cases["c"]["ranks_failed"] == []  # later cases still ran
    assert cases["b"]["ranks_failed"] == [rank_failed] and cases["b"]["bitwise"] is False
    if inject.startswith("raise"):
        assert "injected" in cases["b"]["errors"][str(rank_failed)]  # JSON object keys are strings
    assert not [ln for ln in out[1][1].splitlines() if ln.startswith("{")]  # only rank 0 prints the line


@pytest.mark.parametrize("inject,rank_failed", [("", None), ("corrupt_rank1", 1), ("raise_run_rank1", 1)])
def test_check_gate_at_eight_ranks(inject, rank_failed):
    """The driver's 8-GPU node: the same gate with a world of 8 (reference rule
    2x4, 8x1 and 1x8 cases) -- one failing rank stops all eight before timing."""
    out = _run(inject, world=8)
    if rank_failed is None:
        for rc, o, e in out:
            assert rc == 0, e
            assert "PASSED_GATE" in o
        return
    for rc, o, e in out:
        assert rc == _bench_const("CHECK_FAILED_EXIT"), e
        assert "PASSED_GATE" not in o
    lines = [ln for ln in out[0][1].splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[0][1]
    d = json.loads(lines[0])
    assert d["value"] is None and d["n_gpus"] == 8
    assert d["multi_rank_check"]["cases"]["b"]["ranks_failed"] == [rank_failed]
    for r in range(1, 8):
        assert not [ln for ln in out[r][1].splitlines() if ln.startswith("{")]
