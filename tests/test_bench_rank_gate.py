"""bench.py's _RankGate (CPU, gloo worlds of 2 and 8): when one rank raises inside a
host-side phase of a multi-rank aux measurement, EVERY rank raises at the
same gate -- nobody is left blocked in the next collective -- and the engine
that rank holds is closed.  Stand-in engines: the control flow is under test,
not the kernels."""
from __future__ import annotations

import os
import socket
import subprocess
import sys

import pytest

from conftest import PKG, ROOT

WORKER = r'''
import os, sys
sys.path[:0] = [{root!r}, {pkg!r}]
import torch.distributed as dist
import bench

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
fail_stage, fail_rank = os.environ["FAIL_STAGE"], int(os.environ["FAIL_RANK"])
dist.init_process_group("gloo", rank=rank, world_size=world)


class Eng:
    closed = False

    def close(self):
        Eng.closed = True


def maybe_fail(stage):
    if stage == fail_stage and rank == fail_rank:
        raise ValueError(f"injected in {{stage}}")
    return stage


g = bench._RankGate("aux test", True)
reached = []
try:
    def setup():
        g.engine = Eng()
        return maybe_fail("setup")
    g.run(setup)
    g.gate("setup")
    reached.append("setup")
    g.run(lambda: maybe_fail("timed"))
    g.gate("timed")
    reached.append("timed")
    print(f"OK {{rank}} {{reached}}", flush=True)
except RuntimeError as exc:
    print(f"RAISED {{rank}} {{reached}} closed={{Eng.closed}} :: {{exc}}", flush=True)
dist.barrier()   # every rank reaches the same point afterwards
dist.destroy_process_group()
'''


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("world,stage,fail_rank", [(2, "setup", 1), (2, "timed", 0), (2, "timed", 1), (2, "none", 0),
                                                    # the driver's 8-GPU node: one rank of eight fails
                                                    (8, "setup", 5), (8, "timed", 7), (8, "none", 0)])
def test_rank_gate_all_ranks_raise_together(tmp_path, world, stage, fail_rank):
    script = tmp_path / "w.py"
    script.write_text(WORKER.format(root=str(ROOT), pkg=str(PKG)))
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   FAIL_STAGE=stage, FAIL_RANK=str(fail_rank), OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=120) for p in procs]
    for p, (out, err) in zip(procs, outs):
        assert p.returncode == 0, err
    lines = [out.strip().splitlines()[-1] for out, _ in outs]
    if stage == "none":
        assert all(line.startswith("OK") and "'timed'" in line for line in lines), lines
        return
    want = "[]" if stage == "setup" else "['setup']"
    for r, line in enumerate(lines):
        assert line.startswith(f"RAISED {r} {want} closed=True"), lines
        assert ("this rank" in line) == (r == fail_rank), lines
