"""The resident kernel's residency failure: deterministic, bounded, recoverable.

The lattice-resident persistent kernel (lbm_resident.hip; AUTO's choice for all
four reference grids) needs every tile of its grid on the device at once.  A
tile that is not -- another kernel holds its CU -- never publishes, so its
neighbours' polls hit the deadline, set the status word and the grid drains.
The engine then repeats the run on the STEP2 kernel from the untouched input
lattice and keeps STEP2 for the handle (lbm_engine.hip run_steps), so
lbm_run keeps the blocking engine.run(1) contract of the reference host
(/root/reference/main/LbmRunner.cpp:102-104) whatever else runs on the GPU.

Failure injection (debug knobs, read only with LBM_DEBUG_KNOBS=1):
  * LBM_DEBUG_RES_STALL_TILE / _STEP: one tile leaves its step loop without
    publishing -- a residency failure on every launch mode, every time;
  * LBM_DEBUG_RES_OVERSUBSCRIBE: a grid with more tiles than the device holds
    (the cooperative launch is refused, the plain one times out);
  * LBM_DEBUG_RES_TIMEOUT_MS shortens the 2 s poll deadline.
And without injection: the reference run beside another handle that keeps the
device busy.  Every result is compared bitwise with the CPU oracle.
"""
from __future__ import annotations

import hashlib
import threading
import time

import numpy as np
import pytest

from conftest import load_problem, oracle_manifest
from lbm_amd import io as lio
from oracle import oracle

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("debug_knobs")]

# av_vels: the oracle sums |u| of 262 144 cells sequentially in fp32, the GPU in
# fixed-order trees (the lattices are compared bitwise)
AV_RTOL = 1e-4


def sha(cells):
    return hashlib.sha256(np.ascontiguousarray(cells, dtype="<f4").tobytes()).hexdigest()


def _problem(n=512, seed=7):
    p = lio.Params(n, n, 0, 10, 0.1, 0.005, 1.85)
    obst = np.zeros((n, n), np.uint8)
    obst[0, :] = obst[-1, :] = 1
    obst[n // 4:3 * n // 4, n // 3] = 1
    rng = np.random.default_rng(seed)
    cells0 = (lio.init_cells(p) * (1 + 0.05 * rng.standard_normal((n, n, 9)))).astype(np.float32)
    return p, obst, cells0


@pytest.mark.parametrize("coop", ["1", "0"])
@pytest.mark.parametrize("flags", [0, 4])  # bitwise, LBM_FLAG_TOLERANCE
def test_stalled_tile_falls_back_bitwise(gpu_lib, coop, flags, monkeypatch):
    """A tile that stops at step 3: the run returns LBM_OK within the deadline,
    the lattice and av_vels are those of the oracle (the STEP2 repeat from the
    pre-run lattice, first accelerate included), the handle reports STEP2 and
    bitwise numerics from then on, and a second run continues the state."""
    monkeypatch.setenv("LBM_RES_COOP", coop)
    monkeypatch.setenv("LBM_DEBUG_RES_STALL_TILE", "5")
    monkeypatch.setenv("LBM_DEBUG_RES_STALL_STEP", "3")
    monkeypatch.setenv("LBM_DEBUG_RES_TIMEOUT_MS", "50")
    p, obst, cells0 = _problem()
    steps1, steps2 = 40, 7
    with gpu_lib.Engine(p, obst, flags=flags) as e:
        assert e.kernel_in_use() == "resident"
        e.load_cells(cells0)
        t0 = time.monotonic()
        e.run_steps(steps1, accelerate_first=True)
        wall = time.monotonic() - t0
        assert wall < 5.0, f"recovery took {wall:.2f} s"
        assert e.kernel_in_use() == "step2"
        assert e.numerics() == "bitwise"
        assert e.run_stats() == (steps1 // 2, 0)
        c1, av1 = e.store(n_av=steps1)
        e.run_steps(steps2)
        c2, av2 = e.store(n_av=steps2)
    ref1, ref_av1 = oracle.run(p, obst, steps1, cells0)
    assert np.array_equal(c1, ref1)
    np.testing.assert_allclose(av1, ref_av1, rtol=AV_RTOL)
    ref2, ref_av2 = oracle.run(p, obst, steps2, ref1, accelerate_first=False)
    assert np.array_equal(c2, ref2)
    np.testing.assert_allclose(av2, ref_av2, rtol=AV_RTOL)


def test_stall_without_knob_gate_is_ignored(gpu_lib, monkeypatch):
    """Product mode (LBM_DEBUG_KNOBS unset): the stall knob is ignored."""
    monkeypatch.delenv("LBM_DEBUG_KNOBS", raising=False)
    monkeypatch.setenv("LBM_DEBUG_RES_STALL_TILE", "0")
    monkeypatch.setenv("LBM_DEBUG_RES_TIMEOUT_MS", "1")
    p, obst, cells0 = _problem(256)
    with gpu_lib.Engine(p, obst) as e:
        e.load_cells(cells0)
        e.run_steps(12, accelerate_first=True)
        assert e.kernel_in_use() == "resident"
        cells, _ = e.store(n_av=12)
    ref, _ = oracle.run(p, obst, 12, cells0)
    assert np.array_equal(cells, ref)


@pytest.mark.parametrize("coop", ["1", "0"])
def test_oversubscribed_grid_falls_back(gpu_lib, coop, monkeypatch, capfd):
    """A resident grid larger than the device holds at once (1024^2 in 128x4
    tiles: 2048 workgroups, about three per CU fit): the cooperative launch is
    refused by the runtime, the plain launch's resident part times out while
    the rest waits -- both end on STEP2 with the oracle's lattice."""
    monkeypatch.setenv("LBM_RES_COOP", coop)
    monkeypatch.setenv("LBM_DEBUG_RES_OVERSUBSCRIBE", "1")
    monkeypatch.setenv("LBM_RES_TH", "4")
    monkeypatch.setenv("LBM_DEBUG_RES_TIMEOUT_MS", "100")
    p, obst = load_problem("1024x1024", iters=30)
    cells0 = lio.init_cells(p)
    with gpu_lib.Engine(p, obst) as e:
        assert e.kernel_in_use() == "resident"
        e.load_cells(cells0)
        t0 = time.monotonic()
        e.run()
        wall = time.monotonic() - t0
        assert e.kernel_in_use() == "step2"
        cells, av = e.store()
    assert "hand-off timed out" in capfd.readouterr().err
    print(f"coop={coop}: oversubscribed grid fell back to step2 in {wall:.3f} s")
    assert wall < 10.0
    ref, ref_av = oracle.run(p, obst, 30, cells0)
    assert np.array_equal(cells, ref)
    np.testing.assert_allclose(av, ref_av, rtol=AV_RTOL)


def test_reference_run_beside_a_busy_handle(gpu_lib):
    """BASELINE config 2 (1024^2, 20 000 steps, AUTO = resident) on a thread while
    another handle keeps the device busy with 8192^2 stream launches: the final
    lattice is the oracle's (manifest sha256) whether the resident grid stayed
    co-resident or the run fell back to STEP2."""
    p, obst = load_problem("1024x1024")
    m = oracle_manifest("1024x1024")
    out = {}

    def reference_run():
        with gpu_lib.Engine(p, obst) as e:
            e.load_cells(lio.init_cells(p))
            e.run()
            out["cells"], out["av"] = e.store()
            out["kernel"] = e.kernel_in_use()

    n = 8192
    pb = lio.Params(n, n, 0, 10, 0.1, 0.005, 1.85)
    ob = np.zeros((n, n), np.uint8)
    ob[0, :] = ob[-1, :] = 1
    with gpu_lib.Engine(pb, ob, flags=gpu_lib.FLAG_TOLERANCE) as busy:
        busy.init_equilibrium()
        busy.run_steps(10)
        th = threading.Thread(target=reference_run)
        th.start()
        while th.is_alive():
            busy.run_steps(200)
        th.join()
    print(f"1024^2 reference run beside the busy handle finished on {out['kernel']}")
    assert sha(out["cells"]) == m["final_f_sha256"]
