"""Product mode: a handle created without LBM_DEBUG_KNOBS ignores stray knobs.

The library reads its tuning and debug knobs only when
LBM_DEBUG_KNOBS=1.  Here the gate is unset and a set of stray knobs that would
change the kernel, the steps per launch, the launch form or the resident
variant sits in the environment: every handle must pick the same kernel and
steps per launch, and produce the same lattice bit for bit, as in a clean
environment (where, in bitwise mode, it also equals the CPU oracle).
"""
from __future__ import annotations

import numpy as np
import pytest

from lbm_amd import io as lio
from oracle import oracle

pytestmark = pytest.mark.gpu

STRAY = {
    "LBM_KERNEL": "vec4", "LBM_STREAM_S": "3", "LBM_TOL_S": "4", "LBM_STREAM_CFG": "0", "LBM_TOL_CFG": "0",
    "LBM_RES_V": "1", "LBM_RES_TH": "16", "LBM_RES_COOP": "0", "LBM_TWO_STEP": "0", "LBM_STREAM_GUIDE": "0",
    "LBM_STREAM_OW16": "0", "LBM_PLACEMENT_TRIES": "1", "LBM_DEBUG_RES_STALL_TILE": "0",
    "LBM_DEBUG_RES_TIMEOUT_MS": "1", "LBM_GRAPH_STEPS": "0", "LBM_XOFF": "72",
}


def _problem(n):
    p = lio.Params(n, n, 0, 10, 0.1, 0.005, 1.85)
    obst = np.zeros((n, n), np.uint8)
    obst[0, :] = obst[-1, :] = 1
    obst[:, n // 3] = 1
    rng = np.random.default_rng(n)
    cells0 = (lio.init_cells(p) * (1 + 0.02 * rng.standard_normal((n, n, 9)))).astype(np.float32)
    return p, obst, cells0


def _run(native, p, obst, cells0, steps, flags):
    with native.Engine(p, obst, flags=flags) as e:
        e.load_cells(cells0)
        e.run_steps(steps, accelerate_first=True)
        cells, av = e.store(n_av=steps)
        return e.kernel_in_use(), e.steps_per_launch(), e.run_stats(), e.numerics(), cells, av


@pytest.mark.parametrize("n,flags,kernel,spl", [
    (512, 0, "resident", None),        # AUTO: the lattice-resident kernel (reference grids)
    (512, 4, "resident", None),
    (2048, 0, "stream", 6),            # AUTO: the stream kernel, bitwise S = 6
    (2048, 4, "stream", 10),           # tolerance S = 10
])
def test_stray_knobs_are_ignored(gpu_lib, n, flags, kernel, spl, monkeypatch):
    steps = 23
    p, obst, cells0 = _problem(n)
    monkeypatch.delenv("LBM_DEBUG_KNOBS", raising=False)
    for k in STRAY:
        monkeypatch.delenv(k, raising=False)
    clean = _run(gpu_lib, p, obst, cells0, steps, flags)
    for k, v in STRAY.items():
        monkeypatch.setenv(k, v)
    stray = _run(gpu_lib, p, obst, cells0, steps, flags)
    assert clean[0] == stray[0] == kernel
    if spl is not None:
        assert clean[1] == stray[1] == spl
    assert clean[2] == stray[2] and clean[3] == stray[3]
    assert np.array_equal(clean[4], stray[4]) and np.array_equal(clean[5], stray[5])
    if flags == 0:
        ref, _ = oracle.run(p, obst, steps, cells0)
        assert np.array_equal(clean[4], ref)
