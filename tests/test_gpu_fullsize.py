"""BASELINE configs 4 and 5 in their decomposed (multi-GPU) form, at full size,
on one GPU: every sub-domain lives on device 0 and halos move by device
copies (LOCAL loop-back), which runs the same boundary / exchange / unpack /
interior schedule the RCCL path runs per rank.  The lattice must be bitwise
equal to a single-domain run of the same engine (and finite).

  * 16384^2 (config 4) as 8 sub-domains: the reference's 2x4 blocks
    (partitionForIpus for 8 on a square grid, StructuredGridUtils.hpp:498-522)
    and 8x1 y slabs; 8 steps (one 6-step stream launch + two one-step
    launches, W1 halo, WG refresh) then 6 more (one fused launch);
  * D3Q19 512^3 (config 5) as 8 z slabs against one slab (parity of the 3-D
    model is unpinned upstream: there is no 3-D reference code).

About 20 GB of device memory per lattice pair and up to ~40 GB of host memory
(two full-domain AoS copies) per test.
"""
from __future__ import annotations

import numpy as np
import pytest

from lbm_amd import io as lio

pytestmark = pytest.mark.gpu

N2 = 16384


def _obstacles_2d(n):
    o = np.zeros((n, n), np.uint8)
    o[0, :] = o[-1, :] = 1
    o[:, 0] = o[:, -1] = 1
    o[:, n // 3] = 1
    return o


def _run_2d(native, p, obst, steps=(8, 6), **kw):
    """steps[0] steps (accelerated first), store; steps[1] more, store.  Returns
    both lattices + av_vels and the launch counts of both runs."""
    with native.Engine(p, obst, devices=[0], **kw) as e:
        e.init_equilibrium()
        e.run_steps(steps[0], accelerate_first=True)
        stats = [e.run_stats()]
        a8, av8 = e.store(n_av=steps[0])
        e.run_steps(steps[1])
        stats.append(e.run_stats())
        a14, av14 = e.store(n_av=steps[1])
        kernel = e.kernel_in_use()
        rects = e.local_rects()
    return kernel, rects, (a8, av8), (a14, av14), stats


@pytest.fixture(scope="module")
def single_16384(gpu_lib):
    p = lio.Params(N2, N2, 8, 10, 0.1, 0.005, 1.85)
    obst = _obstacles_2d(N2)
    kernel, rects, s8, s14, _ = _run_2d(gpu_lib, p, obst)
    assert kernel == "stream" and len(rects) == 1
    assert np.isfinite(s14[0][::251, ::241]).all()
    return p, obst, s8, s14


@pytest.mark.parametrize("grid", [(2, 4), (8, 1)], ids=["2x4-reference-rule", "8x1-slabs"])
def test_16384_eight_subdomains_bitwise(gpu_lib, single_16384, grid):
    p, obst, s8, s14 = single_16384
    if grid == (2, 4):
        R, C, _ = gpu_lib.partition(N2, N2, 8)
        assert (R, C) == (2, 4)  # the engine's default for 8 parts is the reference rule
        kw = dict(parts=8)
    else:
        kw = dict(parts=8, grid=grid)
    kernel, rects, d8, d14, _ = _run_2d(gpu_lib, p, obst, **kw)
    assert kernel == "stream" and len(rects) == 8
    assert {(r[2], r[3]) for r in rects} == {(N2 // grid[1], N2 // grid[0])}
    assert np.array_equal(d8[0], s8[0]), "after 8 steps (two fused launches)"
    np.testing.assert_allclose(d8[1], s8[1], rtol=1e-4)
    assert np.array_equal(d14[0], s14[0]), "after 6 more (fused launch + one-step remainder)"
    np.testing.assert_allclose(d14[1], s14[1], rtol=1e-4)
    assert np.isfinite(d14[0][::251, ::241]).all()


TOL_STEPS = (9, 13)  # S = 10: one fused 9-step launch, then 10 + a fused 3-step remainder
TOL_STATS = [(1, 0), (2, 0)]


@pytest.fixture(scope="module")
def single_16384_tolerance(gpu_lib):
    p = lio.Params(N2, N2, 9, 10, 0.1, 0.005, 1.85)
    obst = _obstacles_2d(N2)
    kernel, rects, s9, s22, stats = _run_2d(gpu_lib, p, obst, steps=TOL_STEPS, flags=gpu_lib.FLAG_TOLERANCE)
    assert kernel == "stream" and len(rects) == 1
    assert stats == TOL_STATS
    assert np.isfinite(s22[0][::251, ::241]).all()
    return p, obst, s9, s22


@pytest.mark.parametrize("grid", [(2, 4), (8, 1)], ids=["2x4-reference-rule", "8x1-slabs"])
def test_16384_eight_subdomains_tolerance_bitwise(gpu_lib, single_16384_tolerance, grid):
    """The tolerance plan bench.py publishes for config 4 (S = 10 launches and
    fused remainders), decomposed as the 8-GPU runs decompose it, against its
    single-domain run: the tolerance collision is the same per-cell arithmetic
    everywhere, so the lattices must be bitwise equal."""
    p, obst, s9, s22 = single_16384_tolerance
    kw = dict(parts=8) if grid == (2, 4) else dict(parts=8, grid=grid)
    kernel, rects, d9, d22, stats = _run_2d(gpu_lib, p, obst, steps=TOL_STEPS, flags=gpu_lib.FLAG_TOLERANCE, **kw)
    assert kernel == "stream" and len(rects) == 8
    assert {(r[2], r[3]) for r in rects} == {(N2 // grid[1], N2 // grid[0])}
    assert stats == TOL_STATS
    assert np.array_equal(d9[0], s9[0]), "after 9 steps (one fused 9-step launch)"
    np.testing.assert_allclose(d9[1], s9[1], rtol=1e-4)
    assert np.array_equal(d22[0], s22[0]), "after 13 more (10 + fused 3)"
    np.testing.assert_allclose(d22[1], s22[1], rtol=1e-4)


def test_d3q19_512_eight_slabs_bitwise(gpu_lib):
    n = 512
    p = lio.Params3D(n, n, n, 4, 0.1, 0.001, 1.85)
    obst = lio.channel_obstacles3d(n, n, n)
    outs = {}
    for parts in (1, 8):
        with gpu_lib.Engine3D(p, obst, parts=parts, devices=[0]) as e:
            assert len(e.local_slabs()) == parts
            e.init_equilibrium()
            e.run_steps(3)           # one three-step pass (slabs of 64 planes: three-plane exchange)
            c3, av3 = e.store(n_av=3)
            e.run_steps(4)           # a three-step pass + a one-step launch
            c7, av7 = e.store(n_av=4)
        outs[parts] = (c3, av3, c7, av7)
    one, eight = outs[1], outs[8]
    assert np.array_equal(eight[0], one[0])
    assert np.array_equal(eight[2], one[2])
    np.testing.assert_allclose(eight[1], one[1], rtol=1e-4)
    np.testing.assert_allclose(eight[3], one[3], rtol=1e-4)
    assert np.isfinite(eight[2][::37, ::31, ::29]).all()


@pytest.mark.gpu
def test_d3q19_512_eight_slabs_tolerance_three_step(gpu_lib):
    """BASELINE config 5's shape in tolerance mode: three-step passes on one
    slab (periodic ghost refresh) and on 8 z slabs of 64 planes (three-plane
    exchange per pass, boundary triples first) -- 7 steps = two three-step
    passes + a one-step launch, then 6 more (two passes): bitwise equal lattices,
    finite, mass conserved."""
    n = 512
    p = lio.Params3D(n, n, n, 4, 0.1, 0.001, 1.85)
    obst = lio.channel_obstacles3d(n, n, n)
    outs = {}
    for parts in (1, 8):
        with gpu_lib.Engine3D(p, obst, parts=parts, devices=[0], flags=gpu_lib.FLAG_TOLERANCE) as e:
            e.init_equilibrium()
            e.run_steps(7)
            c7, av7 = e.store(n_av=7)
            e.run_steps(6)
            c13, av13 = e.store(n_av=6)
        outs[parts] = (c7, av7, c13, av13)
    one, eight = outs[1], outs[8]
    assert np.array_equal(eight[0], one[0])
    assert np.array_equal(eight[2], one[2])
    np.testing.assert_allclose(eight[1], one[1], rtol=1e-4)
    np.testing.assert_allclose(eight[3], one[3], rtol=1e-4)
    assert np.isfinite(eight[2][::37, ::31, ::29]).all()
    m0 = float(one[0].sum(dtype=np.float64))
    assert float(one[2].sum(dtype=np.float64)) == pytest.approx(m0, rel=1e-5)
