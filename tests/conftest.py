"""Shared test setup.

Markers: ``gpu`` = needs an MI355X (runs through the C ABI of liblbm_hip.so).
Everything else runs on the CPU (oracle KATs, I/O, partition/halo plan, ABI
symbol checks, gloo multi-rank decomposition).
"""
from __future__ import annotations

import gzip
import io as _io
import json
import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "lbm-graphcore_amd"
GOLD = ROOT / "tests" / "golden"
for p in (str(ROOT), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)

from lbm_amd import io as lio  # noqa: E402

# The library reads its tuning knobs (LBM_STREAM_CFG, LBM_TILE2, ...) only with
# LBM_DEBUG_KNOBS=1; the tests that select variants through them need it.
# Unset knobs keep the product defaults.
os.environ.setdefault("LBM_DEBUG_KNOBS", "1")

GRIDS = ["128x128", "128x256", "256x256", "1024x1024"]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X GPU (HIP path through the C ABI)")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    config.addinivalue_line("markers", "multigpu: needs >= 2 GPUs (skipped otherwise)")


def load_problem(grid: str, iters: int | None = None):
    p = lio.Params.from_file(str(GOLD / "params" / f"input_{grid}.params"))
    obst = lio.read_obstacles(p.nx, p.ny, str(GOLD / "params" / f"obstacles_{grid}.dat"))
    if iters is not None:
        p = p.with_iters(iters)
    return p, obst


def oracle_manifest(grid: str) -> dict:
    return json.loads((GOLD / "oracle" / f"{grid}.json").read_text())


def oracle_av_vels(grid: str) -> np.ndarray:
    return np.load(_io.BytesIO(gzip.decompress((GOLD / "oracle" / f"{grid}.av_vels.npy.gz").read_bytes())))


def small_problems():
    meta = json.loads((GOLD / "small.json").read_text())
    data = np.load(GOLD / "small.npz")
    out = {}
    for name, m in meta.items():
        p = lio.Params(m["nx"], m["ny"], 10, m["reynolds_dim"], m["density"], m["accel"], m["omega"])
        out[name] = (p, data[f"{name}/obstacles"], data[f"{name}/cells0"],
                     {n: (data[f"{name}/cells_after_{n}"], data[f"{name}/av_{n}"]) for n in (1, 2, 10)})
    return out


@pytest.fixture(scope="session")
def gpu_lib():
    """The HIP library with a visible GPU -- fails (never skips) on a GPU run without it."""
    from lbm_amd import native
    lib = native.load_library()
    if native.device_count() < 1:
        pytest.fail("no HIP device visible to liblbm_hip.so; gpu tests need an MI355X")
    return native
