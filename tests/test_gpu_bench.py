"""bench.py's output contract on one GPU (the line the driver parses).

Runs `python bench.py` in a subprocess with a short step count and checks the
one JSON line: the keys and types the driver reads, the roofline and
cpu_baseline objects' shape, and that value / ms_per_step agree.
"""
from __future__ import annotations

import json
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu


def run_bench(*args):
    out = subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], cwd=ROOT, capture_output=True, text=True,
                         timeout=240, check=True)
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def test_bench_json_contract():
    d = run_bench("--steps", "10", "--warmup", "2", "--no-cpu-baseline", "--no-aux")
    for k, t in (("metric", str), ("value", float), ("unit", str), ("n_gpus", int), ("steps", int), ("warmup", int),
                 ("ms_per_step", float), ("higher_is_better", bool), ("scaling", str), ("dtype", str), ("data", str),
                 ("config", dict), ("roofline", dict)):
        assert isinstance(d[k], t), k
    assert d["n_gpus"] == 1 and d["steps"] == 10 and d["warmup"] == 2
    assert d["unit"] == "MLUPS" and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert "vs_baseline" in d and d["vs_baseline"] is None
    assert "workload" in d["config"] and "8192x8192" in d["config"]["workload"]
    r = d["roofline"]
    # the bound is named only where a fraction reaches 0.75 (HBM per pass or by
    # the PMC bytes, VALU issue from the committed PMC profile), else "latency"
    # (DESIGN.md section 7); achieved / peak / frac stay the HBM roofline
    assert r["bound"] in ("hbm", "valu", "latency") and r["unit"] == "GB/s" and r["peak"] == 8000.0
    fr = {"hbm": max(r["frac"], r["frac_counter_bytes"] or 0), "valu": r["frac_valu_issue"] or 0}
    top = max(fr, key=fr.get)
    assert r["bound"] == (top if fr[top] >= 0.75 else "latency"), r   # never "hbm" at 0.41
    assert d["numerics"] in ("bitwise", "tolerance") and (d["numerics"] == "bitwise" or "tolerance" in d)
    assert 0 < r["frac"] < 1 and r["achieved"] == pytest.approx(r["frac"] * r["peak"], rel=1e-3)
    # value (whole-job MLUPS) and ms_per_step describe the same timed region
    assert d["value"] == pytest.approx(8192 * 8192 / (d["ms_per_step"] * 1e-3) / 1e6, rel=2e-3)
    assert d["av_vels_finite"] is True
    c = r["device_copy"]   # live context figure: a copy of the same bytes on this box
    assert 1000 < c["gbs"] < 8000 and c["pass_vs_copy"] == pytest.approx(r["achieved"] / c["gbs"], rel=1e-2)


@pytest.mark.parametrize("tolerance", [False, True])
def test_bench_config2_check_gate(gpu_lib, tolerance):
    """BASELINE config 2 as the bench reports it (aux config2_1024x1024): all
    20 000 steps, then the reference's two-file gate in memory -- passes in
    both numerics, and the final pressure equals the oracle's bit for bit in
    bitwise mode."""
    sys.path.insert(0, str(ROOT))
    import bench
    flags = gpu_lib.FLAG_TOLERANCE if tolerance else 0
    d = bench.aux_1024(gpu_lib.KERNEL_AUTO, flags)
    g = d["check_gate"]
    assert d["steps"] == 20000 and g["passed"], g
    if tolerance:
        assert abs(g["final_state_max_diff_pct"]) < 0.1 and abs(g["av_max_diff_pct"]) < 0.1, g
    else:
        assert g["pressure_max_abs_diff_vs_oracle"] == 0.0, g


def test_bench_bitwise_numerics_line():
    d = run_bench("--steps", "14", "--warmup", "2", "--no-cpu-baseline", "--no-aux", "--numerics", "bitwise")
    assert d["numerics"] == "bitwise" and "tolerance" not in d
    assert d["launches"]["plan"] in ("2 x 6 + 1 x 2 (fused remainder)", "2 x 5 + 1 x 4 (fused remainder)",
                                     "2 x 7", "3 x 4 + 1 x 2 (fused remainder)")
