"""Pin the CPU oracle (test infrastructure) before trusting it.

* Known-answer tests restated from the reference's own unit tests
  (test/codelets/main.cpp:407-483 accelerate, :813-930 collision,
  :932-992 rebound; test/lbm/main.cpp:116-412 periodic shifts).
* The reference's committed golden outputs check/*.dat (gate: check.py's 1 %).
* Bitwise agreement with the reference's own LastChance binary (recorded by
  tests/golden/make_golden.py; re-run here when oracle/_ref exists).
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import (GOLD, load_problem, oracle_av_vels, oracle_manifest, oracle_pressure, reference_final_state,
                      small_problems)
from lbm_amd import check as lcheck
from lbm_amd import io as lio
from oracle import oracle


def P(nx, ny, density=0.1, accel=0.005, omega=1.85, iters=1):
    return lio.Params(nx, ny, iters, 10, density, accel, omega)


def test_accelerate_kat():
    # test/codelets/main.cpp:407-483: nx=3, ny=2, density 9, accel 1 -> w1=1, w2=0.25
    p = P(3, 2, density=9.0, accel=1.0)
    cells = np.array([[1, 0.5, 1, 1, 1, 1, 1, 1, 1], list(range(9)), list(range(9)),
                      list(range(2, 11)), list(range(2, 11)), list(range(2, 11))], np.float32).reshape(2, 3, 9)
    obst = np.array([[0, 1, 0], [0, 1, 1]], np.uint8)
    out = cells.copy()
    oracle.accelerate(p, out, obst)
    w1, w2 = 1.0, 0.25
    assert np.array_equal(out[0, 0], cells[0, 0])  # W - w1 not > 0
    assert np.array_equal(out[0, 1], cells[0, 1])  # obstacle
    exp = np.array([0, 1 + w1, 2, 3 - w1, 4, 5 + w2, 6 - w2, 7 - w2, 8 + w2], np.float32)
    assert np.array_equal(out[0, 2], exp)
    assert np.array_equal(out[1], cells[1])  # only row ny-2


def _uniform(nx, ny, vals):
    return np.broadcast_to(np.asarray(vals, np.float32), (ny, nx, 9)).copy()


VALS = [2.30, 2.31, 2.32, 2.33, 2.34, 2.35, 2.36, 2.37, 2.38]


def _equilibrium(cell, omega=1.0):
    # test/codelets/main.cpp:873-921 textbook equilibrium (c^2 = 1/3)
    cell = np.asarray(cell, np.float64)
    rho = cell.sum()
    ux = (cell[1] + cell[5] + cell[8] - cell[3] - cell[6] - cell[7]) / rho
    uy = (cell[2] + cell[5] + cell[6] - cell[4] - cell[7] - cell[8]) / rho
    u = [0, ux, uy, -ux, -uy, ux + uy, -ux + uy, -ux - uy, ux - uy]
    w = [4 / 9] + [1 / 9] * 4 + [1 / 36] * 4
    usq = ux * ux + uy * uy
    eq = np.array([w[i] * rho * (1 + 3 * u[i] + 4.5 * u[i] ** 2 - 1.5 * usq) for i in range(9)])
    return cell + omega * (eq - cell)


def test_collision_and_rebound_kat():
    # On a uniform lattice streaming is the identity, so one fused step is
    # collision (fluid) / rebound (obstacle): test/codelets/main.cpp:813-992.
    p = P(2, 1, omega=1.0, accel=0.0)
    cells = _uniform(2, 1, VALS)
    obst = np.array([[1, 0]], np.uint8)
    out, tot = oracle.step(p, cells, obst)
    assert np.array_equal(out[0, 0], np.array(VALS, np.float32)[[0, 3, 4, 1, 2, 7, 8, 5, 6]])
    np.testing.assert_allclose(out[0, 1], _equilibrium(VALS), rtol=2e-6)
    ux = (VALS[1] + VALS[5] + VALS[8] - VALS[3] - VALS[6] - VALS[7]) / sum(VALS)
    uy = (VALS[2] + VALS[5] + VALS[6] - VALS[4] - VALS[7] - VALS[8]) / sum(VALS)
    assert tot == pytest.approx(np.hypot(ux, uy), rel=1e-5)


@pytest.mark.parametrize("nx,ny", [(5, 3), (8, 8), (1, 4), (6, 1)])
def test_periodic_streaming_kat(nx, ny):
    # omega = 0 and no acceleration: the step is pure pull streaming, i.e. a
    # periodic roll of each plane by its velocity (cf. DoubleRoll KATs,
    # test/lbm/main.cpp:116-412).
    rng = np.random.default_rng(nx * 100 + ny)
    cells = rng.random((ny, nx, 9), dtype=np.float32) + 0.5
    p = P(nx, ny, omega=0.0, accel=0.0)
    out, _ = oracle.step(p, cells, np.zeros((ny, nx), np.uint8))
    cx = [0, 1, 0, -1, 0, 1, -1, -1, 1]
    cy = [0, 0, 1, 0, -1, 1, 1, -1, -1]
    for k in range(9):
        assert np.array_equal(out[..., k], np.roll(cells[..., k], (cy[k], cx[k]), axis=(0, 1))), k


def test_mass_conservation():
    p, obst = load_problem("128x128", iters=50)
    cells0 = oracle.init_cells(p)
    cells, _ = oracle.run(p, obst, 50, cells0)
    assert np.sum(cells, dtype=np.float64) == pytest.approx(np.sum(cells0, dtype=np.float64), rel=1e-5)


def test_ghosted_step_matches_periodic():
    # the ghosted form used by the decomposition tests is the same arithmetic
    p, obst = load_problem("128x256", iters=1)
    rng = np.random.default_rng(7)
    cells = (oracle.init_cells(p) * (1 + 0.01 * rng.standard_normal((p.ny, p.nx, 9)))).astype(np.float32)
    ref, tot = oracle.step(p, cells, obst)
    g = np.pad(cells, ((1, 1), (1, 1), (0, 0)), mode="wrap")
    out, tot2 = oracle.step_ghosted(p, g, obst, p.ny - 2)
    assert np.array_equal(out, ref)
    assert tot2 == tot


def test_small_vectors_reproduce():
    for name, (p, obst, cells0, after) in small_problems().items():
        for n, (cells_n, av_n) in after.items():
            cells, av = oracle.run(p, obst, n, cells0)
            assert np.array_equal(cells, cells_n), (name, n)
            assert np.array_equal(av, av_n), (name, n)


@pytest.mark.parametrize("grid", ["128x128", "128x256"])
def test_oracle_matches_reference_fixtures(grid, tmp_path):
    # full run (40 000 steps, ~10-20 s) against the reference's check/*.dat at check.py's 1 %
    p, obst = load_problem(grid)
    cells, av = oracle.run(p, obst)
    lio.write_average_velocities(str(tmp_path / "av.dat"), av)
    lio.write_results(str(tmp_path / "fs.dat"), p, obst, cells)
    res = lcheck.compare(GOLD / "check" / f"{grid}.av_vels.dat.gz", GOLD / "check" / f"{grid}.final_state.dat.gz",
                         tmp_path / "av.dat", tmp_path / "fs.dat", 1.0)
    assert res["passed"], res
    assert abs(res["av"]["max_diff_pcnt"]) < 0.2 and abs(res["fs"]["max_diff_pcnt"]) < 0.1
    m = oracle_manifest(grid)
    from golden.make_golden import lattice_sha256
    assert lattice_sha256(cells) == m["final_f_sha256"]
    assert np.array_equal(av, oracle_av_vels(grid))
    # the committed final_state pressure fixture is this lattice's pressure column
    _, _, _, pr = lio.macroscopic(p, obst, cells)
    assert np.array_equal(pr, oracle_pressure(grid))


@pytest.mark.parametrize("grid", ["128x128", "128x256", "256x256", "1024x1024"])
def test_final_state_fixture_gate(grid, tmp_path):
    """The second file of the two-file gate on every grid.  Where the reference
    ships check/<grid>.final_state.dat, the oracle's pressure fixture passes
    check.py against it; everywhere, the fixture's sha256 is the manifest's."""
    import hashlib
    pr = oracle_pressure(grid)
    m = oracle_manifest(grid)
    assert pr.dtype == np.float32 and pr.shape == (m["ny"], m["nx"])
    assert hashlib.sha256(pr.tobytes()).hexdigest() == m["final_state_pressure_sha256"]
    ref_fs, src = reference_final_state(grid)
    if src == "reference check/":
        ref = lcheck.load_final_state(ref_fs)
        d = lcheck.diff_values(ref[:, 2], pr.ravel().astype(np.float64))
        assert abs(d["max_diff_pcnt"]) < 0.1, d
    else:
        assert grid in ("256x256", "1024x1024")


@pytest.mark.parametrize("grid", ["128x128", "128x256", "256x256", "1024x1024"])
def test_manifest_pinned_to_reference(grid):
    """The committed manifests record the oracle vs the reference binary and vs check/*.dat."""
    m = oracle_manifest(grid)
    if "reference_binary" in m:
        assert m["reference_binary"]["av_vels_identical"], m
        assert m["reference_binary"]["final_state_identical"], m
    ref_av = lcheck.load_av_vels(GOLD / "check" / f"{grid}.av_vels.dat.gz")
    d = lcheck.diff_values(ref_av, oracle_av_vels(grid).astype(np.float64))
    assert abs(d["max_diff_pcnt"]) < 0.2


def test_oracle_vs_reference_binary_short(tmp_path):
    """Bitwise text identity with the reference's own LastChance (only where it was built)."""
    if not oracle.REF_LASTCHANCE.exists():
        pytest.skip("oracle/_ref/lastchance not built (reference sources absent)")
    pf = tmp_path / "p.params"
    pf.write_text("128\n128\n500\n10\n0.1\n0.005\n1.85\n")
    of = GOLD / "params" / "obstacles_128x128.dat"
    ref = oracle.run_reference(str(pf), str(of), str(tmp_path))
    p = lio.Params.from_file(str(pf))
    obst = lio.read_obstacles(p.nx, p.ny, str(of))
    cells, av = oracle.run(p, obst)
    ours = "".join(f"{i}:\t{float(v):.12E}\n" for i, v in enumerate(av))
    assert open(ref["av_vels"]).read() == ours
    assert ref["reynolds"] == pytest.approx(oracle.reynolds(p, oracle.av_velocity(p, cells, obst)), rel=1e-6)


# ---------------------------------------------- unfused pipeline oracle ----

def test_pipe_collision_kat():
    """Textbook BGK (CollisionVertex, D2Q9CodeletsOptimised.cpp:150-205) on one fluid
    cell next to an obstacle cell (rebound): the collision part matches the KAT's
    float64 equilibrium (test/codelets/main.cpp:873-921) to fp32 rounding."""
    p = P(2, 1, accel=0.0, omega=1.0)
    cells = _uniform(2, 1, VALS)
    obst = np.array([[1, 0]], np.uint8)
    out, _ = oracle.pipe_run(p, obst, 1, cells)
    assert np.array_equal(out[0, 0], np.asarray(VALS, np.float32)[[0, 3, 4, 1, 2, 7, 8, 5, 6]])
    np.testing.assert_allclose(out[0, 1], _equilibrium(VALS, 1.0), rtol=2e-6)


def test_pipe_oracle_close_to_fused():
    """The two schemes differ only in when the accelerate is applied and in the
    collision's expression form: after 200 steps the states agree closely."""
    p, obst = load_problem("128x128", iters=200)
    a, av_a = oracle.run(p, obst, 200)
    b, av_b = oracle.pipe_run(p, obst, 200)
    np.testing.assert_allclose(b, a, rtol=1e-2, atol=1e-4)  # row ny-2 differs most (accelerate timing)
    np.testing.assert_allclose(av_b, av_a, rtol=5e-2)


def test_pipe_oracle_reference_gate_128():
    """Full 40 000-step 128x128 run of the pipeline restatement: reproduces its
    committed manifest bit for bit and passes check.py against the reference's
    own check/128x128.*.dat fixtures (the pin for this scheme)."""
    import hashlib
    import json
    p, obst = load_problem("128x128")
    cells, av = oracle.pipe_run(p, obst)
    m = json.loads((GOLD / "oracle_pipe" / "128x128.json").read_text())
    assert hashlib.sha256(np.ascontiguousarray(cells, "<f4").tobytes()).hexdigest() == m["final_f_sha256"]
    assert m["check_py"]["passed"]
    ref = lcheck.load_av_vels(GOLD / "check" / "128x128.av_vels.dat.gz")
    d = lcheck.diff_values(ref, av.astype(np.float64))
    assert abs(d["max_diff_pcnt"]) < 1.0


def test_oracle_mt_bitwise():
    """The OpenMP restatement (all-cores CPU baseline) gives the same lattice."""
    p, obst = load_problem("128x256", iters=40)
    a, av_a = oracle.run(p, obst, 40)
    b, av_b = oracle.run_mt(p, obst, 40, 4)
    assert np.array_equal(a, b)
    np.testing.assert_allclose(av_b, av_a, rtol=1e-4)  # row-wise partial sums


def test_reference_binary_all_obstacles_and_single_column(tmp_path):
    """The degenerate inputs tests/test_gpu_edge.py runs on the GPU, through
    the reference's own LastChance: every cell an obstacle gives av_vels of
    0 / 0 free cells -- NaN -- as the oracle does; a single-column channel
    (nx = 1, periodic onto itself) matches the oracle's av_vels text exactly."""
    if not oracle.REF_LASTCHANCE.exists():
        pytest.skip("oracle/_ref/lastchance not built (reference sources absent)")
    pf, of = tmp_path / "a.params", tmp_path / "a.dat"
    pf.write_text("16\n8\n10\n10\n0.1\n0.005\n1.85\n")
    of.write_text("".join(f"{x} {y} 1\n" for y in range(8) for x in range(16)))
    (tmp_path / "a").mkdir()
    ref = oracle.run_reference(str(pf), str(of), str(tmp_path / "a"))
    ref_av = lcheck.load_av_vels(ref["av_vels"])
    p = lio.Params.from_file(str(pf))
    _, av = oracle.run(p, lio.read_obstacles(p.nx, p.ny, str(of)))
    assert ref_av.size == 10 and np.isnan(ref_av).all() and np.isnan(av).all()
    pf2, of2 = tmp_path / "c.params", tmp_path / "c.dat"
    pf2.write_text("1\n12\n40\n10\n0.1\n0.005\n1.85\n")
    of2.write_text("0 0 1\n0 11 1\n")
    (tmp_path / "c").mkdir()
    ref = oracle.run_reference(str(pf2), str(of2), str(tmp_path / "c"))
    p2 = lio.Params.from_file(str(pf2))
    _, av2 = oracle.run(p2, lio.read_obstacles(p2.nx, p2.ny, str(of2)))
    assert open(ref["av_vels"]).read() == "".join(f"{i}:\t{float(v):.12E}\n" for i, v in enumerate(av2))
