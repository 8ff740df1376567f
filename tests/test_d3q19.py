"""D3Q19 extension (BASELINE config 5) -- parity UNPINNED
with respect to the reference, which has no 3-D code.

What pins it instead:
* CPU: the restatement (oracle/lbm_oracle3d.c) reproduces the analytic
  Poiseuille profile between bounce-back wall planes, conserves mass, and
  keeps a z-mirror-symmetric state symmetric;
* GPU (through the C ABI, include/lbm3d_hip.h): the HIP lattice is BITWISE
  equal to the restatement -- one slab, z slabs on one GPU (device-copy
  halos), and the RCCL exchange path (one rank sending its faces to itself).
"""
from __future__ import annotations

import numpy as np
import pytest

from lbm_amd import io as lio
from oracle import oracle

pytestmark = pytest.mark.usefixtures("debug_knobs")  # the GPU tests select pass forms by knob

CX = np.array([0, 1, -1, 0, 0, 1, -1, 1, -1, 0, 1, -1, 0, 0, 0, -1, 1, 0, 0])
CY = np.array([0, 0, 0, 1, -1, 1, -1, -1, 1, 0, 0, 0, 1, -1, 0, 0, 0, -1, 1])
CZ = np.array([0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1])
OPP = np.array([0, 2, 1, 4, 3, 6, 5, 8, 7, 14, 15, 16, 17, 18, 9, 10, 11, 12, 13])


def test_velocity_set():
    for k in range(19):
        assert (CX[OPP[k]], CY[OPP[k]], CZ[OPP[k]]) == (-CX[k], -CY[k], -CZ[k])
    assert sorted(zip(CX, CY, CZ)) == sorted({(x, y, z) for x in (-1, 0, 1) for y in (-1, 0, 1)
                                              for z in (-1, 0, 1) if abs(x) + abs(y) + abs(z) <= 2})
    assert list(np.nonzero(CZ == 1)[0]) == [9, 10, 11, 12, 13]     # one contiguous halo block per face
    assert list(np.nonzero(CZ == -1)[0]) == [14, 15, 16, 17, 18]


def test_oracle3d_equilibrium_moments():
    p = lio.Params3D(3, 4, 5, 0, 0.7, 0.0, 1.0)
    c = oracle.init_cells3d(p)
    np.testing.assert_allclose(c.sum(-1), 0.7, rtol=1e-6)
    assert np.all((c * CX).sum(-1) == 0) and np.all((c * CY).sum(-1) == 0) and np.all((c * CZ).sum(-1) == 0)


def test_oracle3d_poiseuille():
    """Body force between wall planes y = 0, ny-1 -> steady parabolic u_x(y) with the
    walls half way between the wall and the first fluid node (bounce-back)."""
    nx, ny, nz = 4, 18, 4
    p = lio.Params3D(nx, ny, nz, 0, 1.0, 1e-5, 1.0)
    cells, _ = oracle.run3d(p, lio.channel_obstacles3d(nx, ny, nz), 6000)
    ux = (cells * CX).sum(-1) / cells.sum(-1)
    nu = (1 / p.omega - 0.5) / 3
    g = p.density * p.accel / 3          # momentum added per step and cell: 2 w1 + 8 w2 = rho a / 3
    y = np.arange(ny)
    ana = g / (2 * nu) * (y - 0.5) * (ny - 1.5 - y)
    prof = ux[:, 1:-1, :]
    assert np.max(np.abs(prof - ana[None, 1:-1, None])) < 1e-2 * ana.max()
    assert np.ptp(prof, axis=(0, 2)).max() < 1e-9   # invariant in x and z


def test_oracle3d_mass_conservation_and_symmetry():
    nx, ny, nz = 6, 7, 8
    p = lio.Params3D(nx, ny, nz, 0, 0.1, 0.0, 1.7)
    rng = np.random.default_rng(3)
    obst = lio.channel_obstacles3d(nx, ny, nz)
    obst[2:6, 3, 2] = 1
    c0 = (oracle.init_cells3d(p) * (1 + 0.02 * rng.standard_normal((nz, ny, nx, 19)))).astype(np.float32)
    # z-mirror symmetric start: state(z) = mirror(state(nz-1-z)) with c_z flipped
    zflip = np.array([k if CZ[k] == 0 else OPP[k] if CX[k] == 0 and CY[k] == 0 else
                      [j for j in range(19) if (CX[j], CY[j], CZ[j]) == (CX[k], CY[k], -CZ[k])][0]
                      for k in range(19)])
    c0 = 0.5 * (c0 + c0[::-1][..., zflip])
    obst = np.maximum(obst, obst[::-1])
    m0 = c0.sum(dtype=np.float64)
    c, _ = oracle.run3d(p, obst, 50, c0)
    assert c.sum(dtype=np.float64) == pytest.approx(m0, rel=1e-6)
    np.testing.assert_allclose(c, c[::-1][..., zflip], rtol=1e-4, atol=1e-7)


# ------------------------------------------------------------------ GPU ----

def _problem(nx, ny, nz, seed, accel=0.002):
    p = lio.Params3D(nx, ny, nz, 0, 0.1, accel, 1.7)
    rng = np.random.default_rng(seed)
    obst = lio.channel_obstacles3d(nx, ny, nz)
    obst[rng.random((nz, ny, nx)) < 0.05] = 1
    c0 = (oracle.init_cells3d(p) * (1 + 0.02 * rng.standard_normal((nz, ny, nx, 19)))).astype(np.float32)
    return p, obst, c0


def _gpu3d(native, p, obst, c0, steps, **kw):
    with native.Engine3D(p, obst, **kw) as e:
        e.load_cells(c0)
        e.run_steps(steps)
        cells, av = e.store(n_av=steps)
        assert e.total_free_cells() == int((obst == 0).sum())
    return cells, av


@pytest.mark.gpu
@pytest.mark.parametrize("pair,two,seg", [("1", "0", "32"), ("0", "0", "32"), ("1", "1", "32"), ("1", "1", "2"),
                                          ("0", "1", "1")])
@pytest.mark.parametrize("nx,ny,nz", [(13, 9, 7), (64, 8, 5), (1, 5, 3), (130, 3, 2), (2, 6, 3), (256, 5, 9),
                                      (138, 7, 6), (61, 17, 1), (125, 10, 4)])
def test_d3q19_bitwise_single_slab(gpu_lib, nx, ny, nz, pair, two, seg, monkeypatch):
    """Column-pair kernel (even nx) and one-cell kernel, and the two-steps-per-pass
    kernel (z segments of 32, 2 and 1 planes; 9 steps = four two-step passes + one
    one-step launch), partial blocks in x, y, z, wrapped tiles (nx < 60).  The
    three-step pass is off here (test_d3q19_three_step_bitwise covers it)."""
    monkeypatch.setenv("LBM3D_THREE", "0")
    monkeypatch.setenv("LBM3D_PAIR", pair)
    monkeypatch.setenv("LBM3D_TWO", two)
    monkeypatch.setenv("LBM3D_SEG", seg)
    p, obst, c0 = _problem(nx, ny, nz, nx + ny + nz)
    ref, ref_av = oracle.run3d(p, obst, 9, c0)
    cells, av = _gpu3d(gpu_lib, p, obst, c0, 9, devices=[0])
    assert np.array_equal(cells, ref)
    np.testing.assert_allclose(av, ref_av, rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("parts", [2, 3, 4, 7])
def test_d3q19_slabs_loopback_bitwise(gpu_lib, parts):
    """z slabs on GPU 0 with device-copy halos (ragged extents), boundary planes on
    their own stream overlapping the interior."""
    p, obst, c0 = _problem(20, 11, 15, parts)
    ref, ref_av = oracle.run3d(p, obst, 12, c0)
    cells, av = _gpu3d(gpu_lib, p, obst, c0, 12, parts=parts, devices=[0])
    assert np.array_equal(cells, ref)
    np.testing.assert_allclose(av, ref_av, rtol=1e-5)


@pytest.mark.gpu
def test_d3q19_rccl_self_exchange_bitwise(gpu_lib):
    """World of one over RCCL: the faces go through ncclSend/ncclRecv to itself."""
    p, obst, c0 = _problem(24, 10, 9, 11)
    ref, ref_av = oracle.run3d(p, obst, 10, c0)
    uid = gpu_lib.rccl_unique_id()
    cells, av = _gpu3d(gpu_lib, p, obst, c0, 10, transport=gpu_lib.TRANSPORT_RCCL, rank=0, world=1, devices=[0],
                       unique_id=uid)
    assert np.array_equal(cells, ref)
    np.testing.assert_allclose(av, ref_av, rtol=1e-5)


@pytest.mark.gpu
def test_d3q19_poiseuille_and_reruns(gpu_lib):
    """Channel flow to steady state in two runs (state carried over): bitwise equal
    to the restatement, and the profile is the analytic parabola."""
    nx, ny, nz = 4, 18, 4
    p = lio.Params3D(nx, ny, nz, 0, 1.0, 1e-5, 1.0)
    obst = lio.channel_obstacles3d(nx, ny, nz)
    ref, _ = oracle.run3d(p, obst, 6000)
    with gpu_lib.Engine3D(p, obst, devices=[0]) as e:
        e.init_equilibrium()
        e.run_steps(2500)
        e.run_steps(3500)
        cells, _ = e.store()
    assert np.array_equal(cells, ref)
    ux = (cells * CX).sum(-1) / cells.sum(-1)
    y = np.arange(ny)
    ana = p.density * p.accel / 3 / (2 * (1 / p.omega - 0.5) / 3) * (y - 0.5) * (ny - 1.5 - y)
    assert np.max(np.abs(ux[:, 1:-1, :] - ana[None, 1:-1, None])) < 1e-2 * ana.max()


@pytest.mark.gpu
def test_d3q19_256cube_steps_and_mass(gpu_lib):
    """256^3 on one GPU: 2 steps bitwise vs the restatement, then mass conserved
    over 50 steps."""
    n = 256
    p = lio.Params3D(n, n, n, 0, 0.1, 0.001, 1.85)
    obst = lio.channel_obstacles3d(n, n, n)
    c0 = oracle.init_cells3d(p)
    ref, ref_av = oracle.run3d(p, obst, 2, c0)
    with gpu_lib.Engine3D(p, obst, devices=[0]) as e:
        e.init_equilibrium()
        e.run_steps(2)
        cells, av = e.store(n_av=2)
        assert np.array_equal(cells, ref)
        # the restatement sums 1.6e7 |u| terms sequentially in fp32, which
        # stagnates once the running sum's ulp nears a term (-7 % here); the GPU
        # sums in trees.  Tight av_vels checks live on the small grids above.
        np.testing.assert_allclose(av, ref_av, rtol=0.1)
        m0 = cells.sum(dtype=np.float64)
        e.run_steps(50)
        cells2, av2 = e.store(n_av=50)
    assert cells2.sum(dtype=np.float64) == pytest.approx(m0, rel=1e-5)
    assert np.all(np.isfinite(av2)) and av2[-1] > av2[0]


@pytest.mark.gpu
def test_d3q19_512cube_64bit_indexing(gpu_lib, monkeypatch):
    """BASELINE config 5's 512^3 on one GPU: 2.55e9 floats per lattice (over 2^31),
    so every index into it must be 64-bit.  3 steps as one three-step pass, as
    one two-step pass plus one pair-kernel step, and as three one-cell steps
    (independent indexing code): bitwise equal, finite."""
    n = 512
    p = lio.Params3D(n, n, n, 0, 0.1, 0.001, 1.85)
    obst = lio.channel_obstacles3d(n, n, n)
    out = {}
    monkeypatch.setenv("LBM3D_PLACEMENT_TRIES", "1")
    for pair, two, three in (("1", "1", "1"), ("1", "1", "0"), ("0", "0", "0")):
        monkeypatch.setenv("LBM3D_PAIR", pair)
        monkeypatch.setenv("LBM3D_TWO", two)
        monkeypatch.setenv("LBM3D_THREE", three)
        with gpu_lib.Engine3D(p, obst, devices=[0]) as e:
            e.init_equilibrium()
            e.run_steps(3)
            out[pair + two + three] = e.store(n_av=3)
    a, av_a = out["111"]
    assert np.isfinite(a[::31, ::29, ::37]).all()
    for key in ("110", "000"):
        b, av_b = out[key]
        assert np.array_equal(a, b), key
        np.testing.assert_allclose(av_a, av_b, rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("parts,seg", [(2, "64"), (3, "4"), (4, "3"), (5, "1"), (8, "64")])
@pytest.mark.parametrize("steps", [8, 9])
def test_d3q19_slabs_two_step_bitwise(gpu_lib, parts, seg, steps, monkeypatch):
    """Two steps per pass on z slabs (BASELINE config 5's 8-slab form): each pass
    computes the two boundary plane pairs first, exchanges them (all 19 speeds of
    two planes each way) and then the interior; odd step counts end with a
    one-step launch.  Ragged slabs of 5..20 planes, z segments of 1..64 planes."""
    monkeypatch.setenv("LBM3D_SEG", seg)
    p, obst, c0 = _problem(22, 9, 40, 100 + parts)
    ref, ref_av = oracle.run3d(p, obst, steps, c0)
    cells, av = _gpu3d(gpu_lib, p, obst, c0, steps, parts=parts, devices=[0])
    assert np.array_equal(cells, ref)
    np.testing.assert_allclose(av, ref_av, rtol=1e-5)
    monkeypatch.setenv("LBM3D_TWO", "0")  # the one-step slab path gives the same lattice
    cells1, _ = _gpu3d(gpu_lib, p, obst, c0, steps, parts=parts, devices=[0])
    assert np.array_equal(cells1, ref)


@pytest.mark.gpu
def test_d3q19_rccl_two_step_self_exchange_bitwise(gpu_lib):
    """World of one over RCCL with the two-step pass: the two-plane ghost pairs go
    through ncclSend / ncclRecv to itself, twice per pass, in the engine's order."""
    p, obst, c0 = _problem(24, 10, 12, 17)
    for steps in (6, 7):
        ref, ref_av = oracle.run3d(p, obst, steps, c0)
        cells, av = _gpu3d(gpu_lib, p, obst, c0, steps, transport=gpu_lib.TRANSPORT_RCCL, rank=0, world=1,
                           devices=[0], unique_id=gpu_lib.rccl_unique_id())
        assert np.array_equal(cells, ref)
        np.testing.assert_allclose(av, ref_av, rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("th,skip,pd", [("12", "0", "0"), ("12", "0", "1")])
@pytest.mark.parametrize("nx,ny,nz,parts", [(64, 8, 5, 1), (125, 23, 9, 1), (61, 17, 3, 1), (70, 31, 24, 3)])
def test_d3q19_two_step_block_rows_bitwise(gpu_lib, nx, ny, nz, parts, th, skip, pd, monkeypatch):
    """The two-step kernel's two load schedules (LBM3D_PD 0: the next plane
    loaded once level 1 is done with the current one, the default; 1: one plane
    prefetched a whole iteration ahead): bitwise vs the oracle on partial and
    wrapped tiles (ny below and above one block's owned rows), one slab and
    z slabs, 9 steps (four passes + one one-step launch)."""
    monkeypatch.setenv("LBM3D_THREE", "0")
    monkeypatch.setenv("LBM3D_TH", th)
    monkeypatch.setenv("LBM3D_SKIP", skip)
    monkeypatch.setenv("LBM3D_PD", pd)
    monkeypatch.setenv("LBM3D_SEG", "4")
    p, obst, c0 = _problem(nx, ny, nz, nx * ny + nz)
    ref, ref_av = oracle.run3d(p, obst, 9, c0)
    cells, av = _gpu3d(gpu_lib, p, obst, c0, 9, parts=parts, devices=[0])
    assert np.array_equal(cells, ref)
    np.testing.assert_allclose(av, ref_av, rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("seg3", ["64", "5", "1"])
@pytest.mark.parametrize("nx,ny,nz", [(13, 9, 7), (64, 8, 5), (1, 5, 3), (130, 3, 2), (61, 17, 1), (125, 23, 9),
                                      (58, 6, 4), (59, 13, 12), (2, 6, 3)])
@pytest.mark.parametrize("skip3", ["1", "0"])
def test_d3q19_three_step_bitwise(gpu_lib, nx, ny, nz, seg3, skip3, monkeypatch):
    """Three steps per pass (step3d_three, single slab, the default there):
    10 steps = three passes + one one-step launch, 8 = two passes + one
    two-step pass; owned tiles of 58 x 6 (partial and wrapped in x and y:
    nx, ny below and above one tile), z segments of 64, 5 and 1 planes, slabs
    thinner than the three ghost planes (nz < 3).  Bitwise vs the oracle, with
    the dead-row skip (LBM3D_SKIP3, the default) and without it."""
    monkeypatch.setenv("LBM3D_THREE", "1")
    monkeypatch.setenv("LBM3D_SKIP3", skip3)
    monkeypatch.setenv("LBM3D_SEG3", seg3)
    p, obst, c0 = _problem(nx, ny, nz, 3 * nx + ny + nz)
    for steps in (10, 8):
        ref, ref_av = oracle.run3d(p, obst, steps, c0)
        cells, av = _gpu3d(gpu_lib, p, obst, c0, steps, devices=[0])
        assert np.array_equal(cells, ref), steps
        np.testing.assert_allclose(av, ref_av, rtol=1e-5)


@pytest.mark.gpu
def test_d3q19_three_step_reruns_and_tolerance(gpu_lib, monkeypatch):
    """The three-step pass across runs (state carried over, ghost planes
    refreshed per pass: 4 + 5 + 6 steps bitwise equal to the oracle's 15),
    and in tolerance mode (6 steps) within 2e-5 relative of the oracle and
    bitwise equal to the two-step passes' tolerance lattice (same per-cell
    arithmetic, other pass structure)."""
    monkeypatch.setenv("LBM3D_THREE", "1")
    p, obst, c0 = _problem(70, 31, 24, 7)
    ref, _ = oracle.run3d(p, obst, 15, c0)
    with gpu_lib.Engine3D(p, obst, devices=[0]) as e:
        e.load_cells(c0)
        for n in (4, 5, 6):
            e.run_steps(n)
        cells, _ = e.store()
    assert np.array_equal(cells, ref)
    # 6 steps: two three-step passes / three two-step passes (a one-step
    # launch would use the bitwise pair kernel in both modes)
    ref6, _ = oracle.run3d(p, obst, 6, c0)
    tol3, _ = _gpu3d(gpu_lib, p, obst, c0, 6, devices=[0], flags=gpu_lib.FLAG_TOLERANCE)
    dev = float(np.max(np.abs(tol3.astype(np.float64) - ref6) / np.maximum(np.abs(ref6), 1e-30)))
    assert dev < 2e-5, dev
    monkeypatch.setenv("LBM3D_THREE", "0")
    tol2, _ = _gpu3d(gpu_lib, p, obst, c0, 6, parts=3, devices=[0], flags=gpu_lib.FLAG_TOLERANCE)
    assert np.array_equal(tol3, tol2)


@pytest.mark.gpu
@pytest.mark.parametrize("parts,seg3", [(2, "64"), (3, "5"), (4, "1"), (6, "64"), (7, "64")])
def test_d3q19_slabs_three_step_bitwise(gpu_lib, parts, seg3, monkeypatch):
    """Three steps per pass on z slabs: the boundary plane triples first, a
    three-plane exchange (all 19 speeds) overlapped with the interior; 10
    steps = three passes + one one-step launch, 8 = two passes + a two-step
    pass.  Ragged slabs of 5..20 planes (7 slabs: some below 6 planes, so the
    engine keeps two-step passes), z segments of 1..64 planes."""
    monkeypatch.setenv("LBM3D_THREE", "1")
    monkeypatch.setenv("LBM3D_SEG3", seg3)
    p, obst, c0 = _problem(22, 9, 40, 200 + parts)
    for steps in (10, 8):
        ref, ref_av = oracle.run3d(p, obst, steps, c0)
        cells, av = _gpu3d(gpu_lib, p, obst, c0, steps, parts=parts, devices=[0])
        assert np.array_equal(cells, ref), steps
        np.testing.assert_allclose(av, ref_av, rtol=1e-5)


@pytest.mark.gpu
def test_d3q19_rccl_three_step_self_exchange_bitwise(gpu_lib, monkeypatch):
    """World of one over RCCL with three-step passes: the three-plane ghost
    triples go through ncclSend / ncclRecv to itself once per pass."""
    monkeypatch.setenv("LBM3D_THREE", "1")
    p, obst, c0 = _problem(24, 10, 12, 19)
    for steps in (6, 7, 8):
        ref, ref_av = oracle.run3d(p, obst, steps, c0)
        cells, av = _gpu3d(gpu_lib, p, obst, c0, steps, transport=gpu_lib.TRANSPORT_RCCL, rank=0, world=1,
                           devices=[0], unique_id=gpu_lib.rccl_unique_id())
        assert np.array_equal(cells, ref), steps
        np.testing.assert_allclose(av, ref_av, rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{}, {"LBM3D_KSPAD": "320"}, {"LBM_LATTICE_PAD": "4096"},
                                 {"LBM_LATTICE_PAD": "1052672", "LBM3D_KSPAD": "64"}])
@pytest.mark.parametrize("two", ["0", "1"])
@pytest.mark.parametrize("nx,ny,nz,parts", [(64, 8, 5, 1), (70, 31, 24, 3)])
def test_d3q19_lattice_placement_bitwise(gpu_lib, nx, ny, nz, parts, two, env, monkeypatch):
    """Lattice placement knobs (padded speed planes, both
    lattices in one allocation): bitwise vs the oracle with
    the one- and two-step kernels, one slab and z slabs."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("LBM3D_TWO", two)
    p, obst, c0 = _problem(nx, ny, nz, nx + ny * nz)
    ref, ref_av = oracle.run3d(p, obst, 7, c0)
    cells, av = _gpu3d(gpu_lib, p, obst, c0, 7, parts=parts, devices=[0])
    bad = np.argwhere(cells != ref)
    assert len(bad) == 0, (len(bad), bad[:8].tolist(), sorted(set(bad[:, 0].tolist())), sorted(set(bad[:, 3].tolist())))
    np.testing.assert_allclose(av, ref_av, rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("parts", [1, 3])
def test_d3q19_tolerance_vs_oracle(gpu_lib, parts):
    """LBM_FLAG_TOLERANCE (cell3dt in the two-step passes): every population
    within 2e-5 relative of the restatement after 8 steps (four two-step
    passes; three-step passes where the slabs allow them), av_vels within 1e-4,
    and the tolerance result does not depend on the slab decomposition (bitwise
    equal to one slab)."""
    p, obst, c0 = _problem(70, 31, 24, 99)
    ref, ref_av = oracle.run3d(p, obst, 8, c0)
    one, _ = _gpu3d(gpu_lib, p, obst, c0, 8, devices=[0], flags=gpu_lib.FLAG_TOLERANCE)
    cells, av = _gpu3d(gpu_lib, p, obst, c0, 8, parts=parts, devices=[0], flags=gpu_lib.FLAG_TOLERANCE)
    dev = float(np.max(np.abs(cells.astype(np.float64) - ref) / np.maximum(np.abs(ref), 1e-30)))
    assert dev < 2e-5, dev
    assert not np.array_equal(cells, ref)  # the flag really selects the other collision
    assert np.array_equal(cells, one)
    np.testing.assert_allclose(av, ref_av, rtol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [0, 4])
@pytest.mark.parametrize("three", ["1", "0"])
def test_d3q19_placement_probe_transparent(gpu_lib, flags, three, monkeypatch):
    """The D3Q19 placement probe (forced on a small slab: LBM3D_PROBE_MIN_CELLS=0,
    three candidate pairs) leaves the engine as a fresh one: bitwise the same
    lattice and av_vels as with the probe off, and (bitwise mode) as the oracle."""
    p, obst, c0 = _problem(70, 31, 24, 5)
    monkeypatch.setenv("LBM3D_THREE", three)  # the probe times the engine's own pass form
    out = []
    for tries in ("1", "3"):
        monkeypatch.setenv("LBM3D_PLACEMENT_TRIES", tries)
        monkeypatch.setenv("LBM3D_PROBE_MIN_CELLS", "0")
        out.append(_gpu3d(gpu_lib, p, obst, c0, 9, devices=[0], flags=flags))
    assert np.array_equal(out[0][0], out[1][0])
    assert np.array_equal(out[0][1], out[1][1])
    if flags == 0:
        ref, _ = oracle.run3d(p, obst, 9, c0)
        assert np.array_equal(out[1][0], ref)


@pytest.mark.gpu
@pytest.mark.parametrize("three", ["1", "0"])
def test_d3q19_tolerance_long_run(gpu_lib, three, monkeypatch):
    """The D3Q19 tolerance collision (cell3dt: one v_rcp_f32 of rho, no Newton
    step since round 5) over 3000 steps of a driven channel with random
    obstacles, three- and two-step passes: every population within 2e-3
    relative of the oracle (the bound stated for the 2-D collision over the full
    reference runs) and av_vels within 2e-3 -- pins the long-run error the
    8-step tests above cannot see (a bias of the reciprocal grows with the run)."""
    monkeypatch.setenv("LBM3D_THREE", three)
    steps = 3000
    p, obst, c0 = _problem(70, 31, 24, 4242)
    ref, ref_av = oracle.run3d(p, obst, steps, c0)
    cells, av = _gpu3d(gpu_lib, p, obst, c0, steps, devices=[0], flags=gpu_lib.FLAG_TOLERANCE)
    dev = float(np.max(np.abs(cells.astype(np.float64) - ref) / np.maximum(np.abs(ref), 1e-30)))
    dav = float(np.max(np.abs(av.astype(np.float64) - ref_av) / np.abs(ref_av)))
    print(f"D3Q19 tolerance {steps} steps (three={three}): populations {dev:.3e}, av_vels {dav:.3e}")
    assert dev < 2e-3, dev
    assert dav < 2e-3, dav
