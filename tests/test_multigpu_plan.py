"""CPU checks of what the multi-GPU paths will run on the first 8-GPU node
(VERDICT r05 item 7): the >= 2-GPU test's case list (tests/multigpu_worker.py
case_list) and bench.py's N > 1 self-check (_check_cases) must cover
BASELINE config 4's decomposition -- 16384^2 over 8 ranks by the reference
partitionForIpus rule (StructuredGridUtils.hpp:498-522) = 2x4 blocks of
4096 x 8192 -- and config 5's 8 z slabs."""
from __future__ import annotations

import sys

import pytest

from conftest import PKG, ROOT, TESTS_DIR  # noqa: F401


def _native():
    from lbm_amd import native
    native.load_library()
    return native


def test_config4_rule_is_2x4_at_eight_ranks():
    native = _native()
    R, C, rects = native.partition(16384, 16384, 8)
    assert (R, C) == (2, 4)
    assert {(w, h) for _, _, w, h in rects} == {(4096, 8192)}


@pytest.mark.parametrize("world", [2, 4, 8])
def test_multigpu_worker_cases_cover_config4_and_config5(world):
    native = _native()
    sys.path.insert(0, str(TESTS_DIR))
    import multigpu_worker
    plan = multigpu_worker.case_list(world)
    R4, C4, rects4 = native.partition(16384, 16384, world)
    c4 = plan["config4"]
    assert tuple(c4["grid"]) == (R4, C4)
    R, C, rects = native.partition(c4["nx"], c4["ny"], world, *c4["grid"])
    # same grid, same block width as config 4; a quarter of its block height
    assert (R, C) == (R4, C4)
    assert {w for _, _, w, _ in rects} == {w for _, _, w, _ in rects4}
    assert {4 * h for _, _, _, h in rects} == {h for _, _, _, h in rects4}
    assert c4["steps"] == 20  # the driver's timed plan: 2 x 10 (tolerance)
    if world == 8:
        assert (R, C) == (2, 4) and {(w, 4 * h) for _, _, w, h in rects} == {(4096, 8192)}
    d3 = plan["d3q19"]
    assert d3["slabs"] == world and d3["nz"] == 8 * world
    # the 2048^2 cases: the reference rule and N x 1 slabs
    g = plan["grids2d"]
    assert (0, 0) in [tuple(x) for x in g["grids"]] and (world, 1) in [tuple(x) for x in g["grids"]]
    if world == 8:
        assert native.partition(g["n"], g["n"], 8)[:2] == (2, 4)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_self_check_covers_config4_blocks(world):
    native = _native()
    sys.path[:0] = [str(ROOT), str(PKG)]
    import bench
    cases = {c[0]: c for c in bench._check_cases(world)}
    name, nx, ny, grid, mode, steps, flags, _ = cases["tolerance_config4_shape"]
    R4, C4, rects4 = native.partition(16384, 16384, world)
    assert tuple(grid) == (R4, C4) and mode == "tolerance" and steps == 20
    _, _, rects = native.partition(nx, ny, world, *grid)
    assert {w for _, _, w, _ in rects} == {w for _, _, w, _ in rects4}
    assert "bitwise_reference_rule" in cases and "bitwise_slabs" in cases
