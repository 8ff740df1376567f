"""GPU end-to-end through the host CLIs (the reference's own entry points):
lbm_runner (LbmRunner.cpp flags) and compare_lbm (LastChance.cpp positional
CLI), gated with the check.py restatement against the reference's
check/*.dat fixtures; plus hipGraph replay parity."""
from __future__ import annotations

import gzip
import json
import re
import subprocess

import numpy as np
import pytest

from conftest import GOLD, PKG, load_problem, oracle_manifest
from lbm_amd import check as lcheck
from lbm_amd import io as lio
from oracle import oracle

pytestmark = pytest.mark.gpu


def _gate(tmp_path, grid):
    return lcheck.compare(GOLD / "check" / f"{grid}.av_vels.dat.gz", GOLD / "check" / f"{grid}.final_state.dat.gz",
                          tmp_path / "av_vels.dat", tmp_path / "final_state.dat", 1.0)


@pytest.mark.parametrize("args", [["-n", "1"], ["-n", "4", "--device", "loopback"],
                                  ["-n", "1", "--graph-steps", "50"], ["-n", "2", "--device", "loopback",
                                                                      "--kernel", "scalar"],
                                  ["-n", "1", "--kernel", "stream", "--spl", "3"],
                                  ["-n", "4", "--device", "loopback", "--kernel", "stream"],
                                  ["-n", "1", "--kernel", "resident"],
                                  ["-n", "2", "--device", "loopback", "--kernel", "pipeline"],
                                  ["-n", "1", "--kernel", "stream", "--tolerance"],
                                  ["-n", "2", "--device", "loopback", "--kernel", "stream", "--tolerance",
                                   "--spl", "8"]])
def test_lbm_runner_128(gpu_lib, tmp_path, args):
    exe = PKG / "build" / "lbm_runner"
    r = subprocess.run([str(exe), "--params", str(GOLD / "params" / "input_128x128.params"),
                        "--obstacles", str(GOLD / "params" / "obstacles_128x128.dat"), "--runs", "1",
                        "--out-dir", str(tmp_path), "--exe", "ignored.poplar", "-d"] + args,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    assert "==done==" in r.stdout and "Reynolds number:" in r.stdout and "MLUPS:" in r.stdout
    if "--kernel" in args:
        assert f"step kernel: {args[args.index('--kernel') + 1]}" in r.stdout
    re_out = float(re.search(r"Reynolds number:\s+(\S+)", r.stdout).group(1))
    if "pipeline" in args:  # the unfused pipeline's own oracle (accelerate every step, textbook BGK)
        m = json.loads((GOLD / "oracle_pipe" / "128x128.json").read_text())
    else:
        m = oracle_manifest("128x128")
    # tolerance mode: the reciprocal collision, within its stated tolerance of the oracle
    assert re_out == pytest.approx(m["reynolds_last_av"], rel=2e-3 if "--tolerance" in args else 2e-4)
    res = _gate(tmp_path, "128x128")
    assert res["passed"], res
    # -d: the per-launch-class device-time summary (LbmRunner.cpp:115-122's profile summary)
    assert "Profile summary" in r.stdout
    if "step kernel: resident" in r.stdout:   # AUTO keeps 128x128 resident on chip
        assert "resident_steps" in r.stdout and "HBM roofline: n/a" in r.stdout
    else:
        assert re.search(r"% of the 8000 GB/s HBM roofline", r.stdout)


def test_lbm_runner_json_record_and_profile(gpu_lib, tmp_path):
    """--json appends one record whose rates agree with the printed ones and
    whose profile classes account for the fused launches of every run."""
    exe = PKG / "build" / "lbm_runner"
    out = tmp_path / "runs.jsonl"
    for _ in range(2):
        r = subprocess.run([str(exe), "--params", str(GOLD / "params" / "input_128x256.params"),
                            "--obstacles", str(GOLD / "params" / "obstacles_128x256.dat"), "--runs", "2",
                            "--out-dir", str(tmp_path), "--kernel", "stream", "--spl", "5", "-d", "--json", str(out)],
                           capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr
    recs = [json.loads(line) for line in out.read_text().splitlines()]
    assert len(recs) == 2
    rec = recs[-1]
    p, _ = load_problem("128x256")
    assert rec["kernel"] == "stream" and rec["steps_per_launch"] == 5 and rec["numerics"] == "bitwise"
    assert rec["steps"] == p.max_iters and rec["hbm_passes_per_run"] == p.max_iters // 5 + (p.max_iters % 5 > 1) + \
        (p.max_iters % 5 == 1)
    printed = float(re.search(r"MLUPS: (\S+)", r.stdout).group(1))
    assert rec["mlups"] == pytest.approx(printed, rel=1e-3)
    assert rec["gbs_per_pass"] == pytest.approx(72 * p.nx * p.ny * rec["hbm_passes_per_run"] / rec["avg_seconds"] / 1e9,
                                                rel=1e-4)
    assert 0 < rec["hbm_roofline_frac"] < 1
    prof = {k["name"]: k for k in rec["profile"]}
    fused = prof["stream_steps2d S=5"]
    assert fused["launches"] == 3 * (p.max_iters // 5)   # three runs: lbm_run + 2 timed
    assert 0 < fused["min_ms"] <= fused["total_ms"] / fused["launches"] <= fused["max_ms"]
    assert prof["accelerate_row"]["launches"] == 3 and prof["finalize_av"]["launches"] == 3


def test_compare_lbm_128x256(gpu_lib, tmp_path):
    exe = PKG / "build" / "compare_lbm"
    r = subprocess.run([str(exe), str(GOLD / "params" / "input_128x256.params"),
                        str(GOLD / "params" / "obstacles_128x256.dat")], capture_output=True, text=True,
                       cwd=tmp_path, timeout=600)
    assert r.returncode == 0, r.stderr
    m = re.search(r"Reynolds number:\s+(\S+)", r.stdout)
    assert float(m.group(1)) == pytest.approx(oracle_manifest("128x256")["reynolds_final_state"], rel=1e-6)
    res = _gate(tmp_path, "128x256")
    assert res["passed"], res
    # LastChance prints %.12E: same format as the reference's fixtures
    first = (tmp_path / "av_vels.dat").read_text().splitlines()[0]
    ref_first = gzip.decompress((GOLD / "check" / "128x256.av_vels.dat.gz").read_bytes()).decode().splitlines()[0]
    assert re.fullmatch(r"0:\t\d\.\d{12}E[-+]\d\d", first) and first.split("\t")[1][:6] == ref_first.split("\t")[1][:6]


@pytest.mark.parametrize("graph_steps", [1, 8, 64])
def test_graph_replay_bitwise(gpu_lib, graph_steps):
    p, obst = load_problem("128x128", iters=301)
    cells0 = lio.init_cells(p)
    # graphs replay the launch-per-step-group kernels (the resident kernel needs none)
    with gpu_lib.Engine(p, obst, graph_steps=graph_steps, kernel=gpu_lib.KERNEL_STEP2) as e:
        e.load_cells(cells0)
        e.run()
        e.run_steps(17)
        cells, av = e.store(n_av=17)
    c1, _ = oracle.run(p, obst, 301, cells0)  # lbm_run: accelerate + 301 steps
    p2 = p.with_iters(17)                       # then 17 plain steps (no accelerate)
    cur = c1.copy()
    avs = []
    free = oracle.free_cells(p, obst)
    for _ in range(17):
        cur, tot = oracle.step(p2, cur, obst)
        avs.append(tot / free)
    assert np.array_equal(cells, cur)
    np.testing.assert_allclose(av, np.array(avs, np.float32), rtol=1e-5)
