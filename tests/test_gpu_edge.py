"""Degenerate inputs on the GPU path (empty and ragged inputs),
each against the CPU oracle (LastChance.cpp:156-267 restated), bitwise:

  * every cell an obstacle: each step is pure bounce-back (out_k = s_opp(k)),
    the lattice must equal the oracle's, and av_vels is 0 / 0 free cells =
    NaN in both (LastChance.cpp:266 with tot_cells = 0; the reference binary
    itself prints NaN there: tests/test_oracle.py) -- every kernel, and the
    tolerance collision, which never runs on such a lattice;
  * a single column (nx = 1), a single row and a single cell: every periodic
    wrap lands on the cell's own row / column;
  * max_iters = 0: lbm_run leaves the lattice as the oracle leaves it and
    writes no av_vels;
  * nx = 0, ny = 0, max_iters < 0: LBM_E_INVALID at create, nothing launched.
"""
from __future__ import annotations

import numpy as np
import pytest

from lbm_amd import io as lio
from oracle import oracle
from test_gpu_parity import SINGLE_MODES, gpu_run, kname, mode_kw

pytestmark = pytest.mark.gpu


def _perturbed(p, seed):
    rng = np.random.default_rng(seed)
    return (lio.init_cells(p) * (1 + 0.05 * rng.standard_normal((p.ny, p.nx, 9)))).astype(np.float32)


@pytest.mark.parametrize("mode", SINGLE_MODES + ["pipeline", "stream10t"])
def test_all_obstacles_bitwise(gpu_lib, mode):
    steps = 13
    p = lio.Params(128, 64, steps, 10, 0.1, 0.005, 1.85)
    obst = np.ones((p.ny, p.nx), np.uint8)
    c0 = _perturbed(p, 5)
    if mode == "pipeline":
        ref, ref_av = oracle.pipe_run(p, obst, steps, c0)
        kw = dict(kernel=gpu_lib.KERNEL_PIPELINE)
    else:
        ref, ref_av = oracle.run(p, obst, steps, c0)
        kw = (dict(kernel=gpu_lib.KERNEL_STREAM, steps_per_launch=10, flags=gpu_lib.FLAG_TOLERANCE)
              if mode == "stream10t" else mode_kw(gpu_lib, mode))
    cells, av, used = gpu_run(gpu_lib, p, obst, c0, steps, **kw)
    assert used == ("stream" if mode == "stream10t" else kname(mode))
    assert np.array_equal(cells, ref), mode
    assert np.isnan(ref_av).all() and np.isnan(av).all(), (mode, av[:4])


@pytest.mark.parametrize("nx,ny", [(1, 8), (8, 1), (1, 1), (2, 1), (1, 2), (3, 5)])
@pytest.mark.parametrize("walls", [False, True])
def test_single_row_column_cell_bitwise(gpu_lib, nx, ny, walls):
    steps = 9
    p = lio.Params(nx, ny, steps, 10, 0.1, 0.005, 1.85)
    obst = np.zeros((ny, nx), np.uint8)
    if walls and nx * ny > 1:
        obst.reshape(-1)[::2] = 1   # every other cell an obstacle
    c0 = _perturbed(p, 11 + nx * 7 + ny)
    ref, ref_av = oracle.run(p, obst, steps, c0)
    cells, av, used = gpu_run(gpu_lib, p, obst, c0, steps)
    assert np.array_equal(cells, ref), used
    both = np.isfinite(ref_av)
    assert np.array_equal(np.isfinite(av), both)
    np.testing.assert_allclose(av[both], ref_av[both], rtol=1e-5)


def test_zero_steps(gpu_lib):
    p = lio.Params(64, 32, 0, 10, 0.1, 0.005, 1.85)
    obst = np.zeros((p.ny, p.nx), np.uint8)
    obst[0, :] = obst[-1, :] = 1
    c0 = _perturbed(p, 3)
    ref, ref_av = oracle.run(p, obst, 0, c0)
    with gpu_lib.Engine(p, obst) as e:
        e.load_cells(c0)
        e.run()
        cells, av = e.store()
    assert len(ref_av) == 0 and len(av) == 0
    assert np.array_equal(cells, ref)


@pytest.mark.parametrize("nx,ny,iters", [(0, 8, 4), (8, 0, 4), (8, 8, -1)])
def test_invalid_sizes_refused(gpu_lib, nx, ny, iters):
    p = lio.Params(nx, ny, iters, 10, 0.1, 0.005, 1.85)
    with pytest.raises(gpu_lib.LbmError) as ei:
        gpu_lib.Engine(p, np.zeros((ny, nx), np.uint8))
    assert ei.value.code == gpu_lib.LBM_E_INVALID
