"""Cross-stream ordering of the multi-sub-domain engines, made deterministic.

The round-4 GPU suite once returned a wrong lattice from
test_pipeline_decomposed_bitwise[2-grid0]: in LOCAL (loop-back) mode the
unpack of step t into a sub-domain's ghost ring did not wait for that
sub-domain's own pack, so when its neighbours ran a step ahead the unpack
could land while the sub-domain's step t-1 propagate was still reading the
ring (lbm_engine.hip exchange(); the fix waits on the receiver's own ev_b).
Such a race shows up once in hundreds of runs.  Here one sub-domain is held
back on purpose: LBM_DEBUG_DELAY_SUB / LBM_DEBUG_DELAY_US queue a spin kernel
(lbm_kernels.hip debug_spin) before each of its compute launches, so every
other sub-domain runs as far ahead as the events allow, every step.

  * with the fix, every kernel stays bitwise equal to its oracle under the
    stall, whichever sub-domain is stalled (2-D: pipeline, scalar, step2,
    stream; D3Q19: one-, two- and three-step passes on z slabs);
  * with the fix switched off (LBM_DEBUG_NO_OWN_WAIT=1, debug only) the
    stalled pipeline run is WRONG -- the stall does expose the race, so the
    passing case above is evidence, not luck.
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import load_problem
from lbm_amd import io as lio
from oracle import oracle

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("debug_knobs")]  # tests select variants by knob

STALL_US = "3000"   # per stalled launch; a 128x256 step of a neighbour takes ~10 us


def _stall(monkeypatch, sub, us=STALL_US, no_own_wait=False):
    monkeypatch.setenv("LBM_DEBUG_DELAY_SUB", str(sub))
    monkeypatch.setenv("LBM_DEBUG_DELAY_US", us)
    monkeypatch.setenv("LBM_DEBUG_NO_OWN_WAIT", "1" if no_own_wait else "0")


def _run2d(native, p, obst, c0, steps, **kw):
    with native.Engine(p, obst, devices=[0], **kw) as e:
        e.load_cells(c0)
        e.run_steps(steps, accelerate_first=True)
        return e.store(n_av=steps)


@pytest.mark.parametrize("parts,grid", [(2, (1, 2)), (2, (2, 1)), (4, (2, 2))])
@pytest.mark.parametrize("sub", [0, 1])
def test_pipeline_stalled_sub_bitwise(gpu_lib, parts, grid, sub, monkeypatch):
    steps = 9
    p, obst = load_problem("128x256", iters=steps)
    c0 = lio.init_cells(p)
    ref, ref_av = oracle.pipe_run(p, obst, steps, c0)
    _stall(monkeypatch, sub)
    cells, av = _run2d(gpu_lib, p, obst, c0, steps, parts=parts, grid=grid, kernel=gpu_lib.KERNEL_PIPELINE)
    assert np.array_equal(cells, ref)
    np.testing.assert_allclose(av, ref_av, rtol=1e-5)


@pytest.mark.parametrize("parts,grid", [(2, (1, 2)), (4, (2, 2))])
def test_pipeline_stall_exposes_missing_wait(gpu_lib, parts, grid, monkeypatch):
    """The control: the same stalled run without the receiver's own wait is
    wrong.  If this ever passes, the stall no longer provokes the race and the
    test above proves nothing."""
    steps = 9
    p, obst = load_problem("128x256", iters=steps)
    c0 = lio.init_cells(p)
    ref, _ = oracle.pipe_run(p, obst, steps, c0)
    _stall(monkeypatch, 0, no_own_wait=True)
    cells, _ = _run2d(gpu_lib, p, obst, c0, steps, parts=parts, grid=grid, kernel=gpu_lib.KERNEL_PIPELINE)
    bad = int(np.sum(cells != ref))
    print(f"{parts} sub-domains, sub 0 stalled, no own wait: {bad} of {ref.size} values differ")
    assert bad > 0


@pytest.mark.parametrize("mode", ["scalar", "step2", "stream3", "stream6"])
@pytest.mark.parametrize("parts,grid,sub", [(2, (1, 2), 0), (2, (1, 2), 1), (4, (2, 2), 0), (4, (2, 2), 2),
                                            (3, (3, 1), 0), (3, (3, 1), 2)])
def test_fused_stalled_sub_bitwise(gpu_lib, mode, parts, grid, sub, monkeypatch):
    """Boundary (high-priority stream) and interior launches of one sub-domain
    each preceded by a stall: the B / X / I event graph alone keeps the
    lattice bitwise equal to the oracle (13 steps: fused launches and, for the
    stream kernel, a fused remainder or a one-step launch)."""
    steps = 13
    p, obst = load_problem("128x256", iters=steps)
    c0 = lio.init_cells(p)
    ref, ref_av = oracle.run(p, obst, steps, c0)
    kw = {"scalar": dict(kernel=gpu_lib.KERNEL_SCALAR, flags=gpu_lib.FLAG_ONE_STEP),
          "step2": dict(kernel=gpu_lib.KERNEL_STEP2),
          "stream3": dict(kernel=gpu_lib.KERNEL_STREAM, steps_per_launch=3),
          "stream6": dict(kernel=gpu_lib.KERNEL_STREAM, steps_per_launch=6)}[mode]
    _stall(monkeypatch, sub, us="1500")
    cells, av = _run2d(gpu_lib, p, obst, c0, steps, parts=parts, grid=grid, **kw)
    assert np.array_equal(cells, ref)
    np.testing.assert_allclose(av, ref_av, rtol=1e-5)


@pytest.mark.parametrize("three", ["0", "1"])
@pytest.mark.parametrize("parts", [2, 3])
@pytest.mark.parametrize("sub", [0, 1])
def test_d3q19_stalled_slab_bitwise(gpu_lib, three, parts, sub, monkeypatch):
    """D3Q19 z slabs in loop-back mode with one slab's boundary and interior
    launches stalled: two- or three-step passes plus a one-step remainder,
    bitwise equal to the 3-D oracle."""
    from test_d3q19 import _gpu3d, _problem
    monkeypatch.setenv("LBM3D_THREE", three)
    _stall(monkeypatch, sub, us="1500")
    p, obst, c0 = _problem(22, 9, 36, 300 + parts)
    steps = 7
    ref, ref_av = oracle.run3d(p, obst, steps, c0)
    cells, av = _gpu3d(gpu_lib, p, obst, c0, steps, parts=parts, devices=[0])
    assert np.array_equal(cells, ref)
    np.testing.assert_allclose(av, ref_av, rtol=1e-5)
