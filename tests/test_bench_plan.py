"""bench.py's choice of steps per launch (CPU only): pick_spl uses the
measured launch times and counts a remainder as the library runs it (one
fused launch of >= 2 steps, include/lbm_hip.h)."""
from __future__ import annotations

import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "lbm-graphcore_amd")]

import bench  # noqa: E402


def test_pick_spl_driver_and_default_runs():
    assert bench.pick_spl(20, 0, "bitwise") == 5        # 4 x 5
    assert bench.pick_spl(20, 0, "tolerance") == 10     # 2 x 10
    assert bench.pick_spl(1000, 0, "bitwise") == 6      # 166 x 6 + 4
    assert bench.pick_spl(1000, 0, "tolerance") == 10   # 100 x 10
    assert bench.pick_spl(20, 4, "tolerance") == 4      # the caller's choice wins


def test_pick_spl_every_step_count_is_valid():
    for numerics, smax in (("bitwise", 6), ("tolerance", 10)):
        for steps in range(0, 200):
            S = bench.pick_spl(steps, 0, numerics)
            assert 2 <= S <= smax


def test_launch_plan_strings():
    assert bench.launch_plan(20, 7, True) == "2 x 7 + 1 x 6 (fused remainder)"
    assert bench.launch_plan(13, 6, True) == "2 x 6 + 1 x 1"
    assert bench.launch_plan(20, 5, True) == "4 x 5"
    assert bench.launch_plan(7, 2, False) == "3 x 2 + 1 x 1"


def test_pick_spl_follows_a_calibration_table():
    """With a measured table (calibrate_launch_ms) the choice follows the box,
    not the LAUNCH_MS fallback."""
    flat = {"ms": {S: 1.0 for S in range(2, 11)}, "one_step_ms": 0.8}
    assert bench.pick_spl(20, 0, "tolerance", table=flat) == 10          # fewest launches
    slow10 = {"ms": {**{S: 1.0 for S in range(2, 10)}, 10: 9.0}, "one_step_ms": 0.8}
    assert bench.pick_spl(20, 0, "tolerance", table=slow10) == 9          # 2 x 9 + a 2-step launch: 3 ms
    assert bench.pick_spl(18, 0, "tolerance", table=slow10) == 9          # 2 x 9
    json_keys = {"ms": {**{str(S): 1.0 for S in range(2, 6)}, "6": 1.4}, "one_step_ms": 0.8}   # keys after a JSON trip
    assert bench.pick_spl(20, 0, "bitwise", table=json_keys) == 5


def test_config2_check_gate_glue(monkeypatch):
    """bench.check_gate_1024 wiring (CPU): fed the oracle's own full-run
    pressure and the reference av_vels it passes with zero difference; a
    perturbed pressure field fails the 1 % gate."""
    import gzip
    import io as _io
    import numpy as np
    from lbm_amd import check as lcheck
    gold = ROOT / "tests" / "golden"
    pr = np.load(_io.BytesIO(gzip.decompress((gold / "oracle" / "1024x1024.final_state_pressure.npy.gz").read_bytes())))
    av = lcheck.load_av_vels(gold / "check" / "1024x1024.av_vels.dat.gz").astype(np.float32)
    monkeypatch.setattr(bench.lio, "macroscopic", lambda p, o, c: (None, None, None, pr))
    g = bench.check_gate_1024(None, None, None, av)
    assert g["passed"] and g["pressure_max_abs_diff_vs_oracle"] == 0.0, g
    bad = pr.copy()
    bad[100, 200] *= 1.05
    monkeypatch.setattr(bench.lio, "macroscopic", lambda p, o, c: (None, None, None, bad))
    g = bench.check_gate_1024(None, None, None, av)
    assert not g["passed"] and abs(g["final_state_max_diff_pct"]) > 1.0, g
