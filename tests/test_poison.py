"""Read-before-write check (SURVEY §5 sanitizer row).

With LBM_POISON=1 both engines fill every fresh device allocation (lattices,
ghost rings, halo buffers, |u| partials, av_local) with all-ones bytes -- a
NaN in every float -- instead of zeros.  Any value an engine reads without
having written it first then reaches the lattice or av_vels as NaN, and the
bitwise comparison with the oracle fails.

The round-2 logs (profiles/r02/placement/dbg_*.log) showed D3Q19 z-slab
two-step engines computing wrong lattices only after engines with
hipDeviceMallocContiguous lattices had been freed in the same process; these
tests rerun the slab shapes of those logs, and the sequence "large engine
created and freed, then a slab engine", with poisoned allocations.
"""
from __future__ import annotations

import numpy as np
import pytest

from lbm_amd import io as lio
from oracle import oracle
import test_d3q19 as T3

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("debug_knobs")]  # tests select variants by knob


@pytest.fixture(autouse=True)
def poisoned(monkeypatch):
    monkeypatch.setenv("LBM_POISON", "1")


@pytest.mark.parametrize("two", ["0", "1"])
@pytest.mark.parametrize("shape", [(70, 31, 24, 3), (64, 8, 5, 1), (38, 12, 20, 4), (70, 31, 24, 1)])
def test_d3q19_poisoned_bitwise(gpu_lib, shape, two, monkeypatch):
    nx, ny, nz, parts = shape
    monkeypatch.setenv("LBM3D_TWO", two)
    p, obst, c0 = T3._problem(nx, ny, nz, nx + ny * nz)
    for steps in (7, 8):
        ref, ref_av = oracle.run3d(p, obst, steps, c0)
        cells, av = T3._gpu3d(gpu_lib, p, obst, c0, steps, parts=parts, devices=[0])
        assert np.array_equal(cells, ref), (shape, two, steps, int((cells != ref).sum()))
        np.testing.assert_allclose(av, ref_av, rtol=1e-5)


def test_d3q19_init_equilibrium_poisoned(gpu_lib):
    """lbm3d_init_equilibrium writes every plane (ghosts included) itself."""
    p, obst, _ = T3._problem(70, 31, 24, 3)
    c0 = oracle.init_cells3d(p)
    ref, _ = oracle.run3d(p, obst, 9, c0)
    with gpu_lib.Engine3D(p, obst, parts=3, devices=[0]) as e:
        e.init_equilibrium()
        e.run_steps(9)
        cells, av = e.store(n_av=9)
    assert np.array_equal(cells, ref)
    assert np.isfinite(av).all()


def test_large_engine_freed_then_slab_engine(gpu_lib):
    """The order-dependence of r02: a large 2-D engine (8192^2 with its
    placement probe: five lattice pairs allocated, four freed, the kept pair
    freed at destroy) and a large D3Q19 engine created and destroyed first,
    then z-slab two-step engines in the same process -- bitwise vs the oracle."""
    n = 8192
    p2 = lio.Params(n, n, 0, 10, 0.1, 0.005, 1.85)
    ob2 = np.zeros((n, n), np.uint8)
    ob2[0, :] = ob2[-1, :] = 1
    with gpu_lib.Engine(p2, ob2) as e:
        e.init_equilibrium()
        e.run_steps(6, accelerate_first=True)
        c, _ = e.store(n_av=6)
        assert np.isfinite(c[::97, ::89]).all()
    del c
    p3 = lio.Params3D(256, 256, 256, 0, 0.1, 0.001, 1.85)
    with gpu_lib.Engine3D(p3, lio.channel_obstacles3d(256, 256, 256), parts=4, devices=[0]) as e:
        e.init_equilibrium()
        e.run_steps(3)
    for shape in ((70, 31, 24, 3), (70, 31, 24, 3), (38, 12, 20, 4)):
        nx, ny, nz, parts = shape
        p, obst, c0 = T3._problem(nx, ny, nz, nx + ny * nz)
        ref, ref_av = oracle.run3d(p, obst, 7, c0)
        cells, av = T3._gpu3d(gpu_lib, p, obst, c0, 7, parts=parts, devices=[0])
        assert np.array_equal(cells, ref), (shape, int((cells != ref).sum()))
        np.testing.assert_allclose(av, ref_av, rtol=1e-5)


@pytest.mark.parametrize("kw", [dict(), dict(parts=4, grid=(2, 2)), dict(parts=3, grid=(1, 3))])
@pytest.mark.parametrize("mode", ["stream5", "step2", "vec4", "resident"])
def test_d2q9_poisoned_bitwise(gpu_lib, kw, mode):
    from test_gpu_parity import mode_kw
    if mode == "resident" and kw:
        pytest.skip("the resident kernel serves one sub-domain")
    rng = np.random.default_rng(7)
    p = lio.Params(312, 260, 11, 10, 0.1, 0.02, 1.7)  # 312: every split keeps widths % 4 == 0 (vec4)
    obst = (rng.random((260, 312)) < 0.03).astype(np.uint8)
    cells0 = (lio.init_cells(p) * (1 + 0.04 * rng.standard_normal((260, 312, 9)))).astype(np.float32)
    ref, ref_av = oracle.run(p, obst, 11, cells0)
    with gpu_lib.Engine(p, obst, devices=[0], **mode_kw(gpu_lib, mode), **kw) as e:
        e.load_cells(cells0)
        e.run_steps(11, accelerate_first=True)
        cells, av = e.store(n_av=11)
    assert np.array_equal(cells, ref)
    np.testing.assert_allclose(av, ref_av, rtol=5e-5)


def test_nonfinite_scan_and_nan_check(gpu_lib, monkeypatch):
    """lbm_nonfinite_count (device NaN / Inf scan) and LBM_NAN_CHECK=1 (every
    run ends with that scan and fails loudly when it finds any)."""
    p = lio.Params(96, 40, 4, 10, 0.1, 0.005, 1.7)
    obst = np.zeros((40, 96), np.uint8)
    obst[0, :] = obst[-1, :] = 1
    cells0 = lio.init_cells(p)
    with gpu_lib.Engine(p, obst, devices=[0]) as e:
        e.load_cells(cells0)
        e.run_steps(4, accelerate_first=True)
        assert e.nonfinite_count() == 0
    bad = cells0.copy()
    bad[17, 33, 5] = np.nan
    bad[3, 90, 0] = np.inf
    monkeypatch.setenv("LBM_NAN_CHECK", "1")
    for kw in (dict(), dict(parts=4, grid=(2, 2))):
        with gpu_lib.Engine(p, obst, devices=[0], **kw) as e:
            e.load_cells(bad)
            assert e.nonfinite_count() == 2
            with pytest.raises(gpu_lib.LbmError) as ei:
                e.run_steps(4, accelerate_first=True)
            assert ei.value.code == gpu_lib.LBM_E_INTERNAL and "LBM_NAN_CHECK" in str(ei.value)
