"""lbm_runner --device cpu (CPU only): the host backend (host/lbm_cpu.hpp,
product code -- it never calls into oracle/) behind the reference's
--device switch (main/LbmRunner.cpp:18; SURVEY.md §5 "Config / flags").

* The lattice is bit-identical to the CPU oracle (LastChance.cpp:192-262
  restated): final_state.dat, printed with %.12e from the lattice, equals the
  oracle's text byte for byte after 1, 2 and 300 steps with any thread count.
* BASELINE config 1 end to end: the full 128x128 reference problem (40 000
  steps) passes the reference gate (check.py, 1 %) against check/*.dat, and
  the Reynolds number (av_vels[maxIters-1], LbmRunner.cpp:129-130) matches the
  oracle manifest's to summation order.
"""
from __future__ import annotations

import json
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLD, PKG
from lbm_amd import check as lcheck
from lbm_amd import io as lio
from oracle import oracle

EXE = PKG / "build" / "lbm_runner"


def _run(tmp_path, params_file, obst_file, threads, runs=0):
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    r = subprocess.run([str(EXE), "--device", "cpu", "--params", str(params_file), "--obstacles", str(obst_file),
                        "--runs", str(runs), "--out-dir", str(tmp_path)], capture_output=True, text=True, env=env,
                       timeout=600)
    assert r.returncode == 0, r.stderr
    return r.stdout


@pytest.mark.parametrize("steps,threads", [(1, 1), (2, 3), (300, 4)])
def test_cpu_device_lattice_bitwise(tmp_path, steps, threads):
    obst_file = GOLD / "params" / "obstacles_128x256.dat"
    base = lio.Params.from_file(str(GOLD / "params" / "input_128x256.params"))
    pf = tmp_path / "p.params"
    pf.write_text(f"{base.nx}\n{base.ny}\n{steps}\n{base.reynolds_dim}\n{base.density}\n{base.accel}\n{base.omega}\n")
    out = _run(tmp_path, pf, obst_file, threads)
    assert "==done==" in out and "host CPU" in out
    p = lio.Params.from_file(str(pf))
    obst = lio.read_obstacles(p.nx, p.ny, str(obst_file))
    cells, av = oracle.run(p, obst, steps, lio.init_cells(p))
    lio.write_results(str(tmp_path / "ref_final_state.dat"), p, obst, cells)
    assert (tmp_path / "final_state.dat").read_bytes() == (tmp_path / "ref_final_state.dat").read_bytes()
    got = lcheck.load_av_vels(tmp_path / "av_vels.dat")
    np.testing.assert_allclose(got, av, rtol=2e-4)  # per-row sums, then rows in order (as the GPU tests: AV_RTOL)


def test_cpu_device_config1_check_py(tmp_path):
    out = _run(tmp_path, GOLD / "params" / "input_128x128.params", GOLD / "params" / "obstacles_128x128.dat", 4,
               runs=1)
    res = lcheck.compare(GOLD / "check" / "128x128.av_vels.dat.gz", GOLD / "check" / "128x128.final_state.dat.gz",
                         tmp_path / "av_vels.dat", tmp_path / "final_state.dat", 1.0)
    assert res["passed"], res
    re_line = [ln for ln in out.splitlines() if ln.startswith("Reynolds number")][0]
    reynolds = float(re_line.split()[-1])
    m = json.loads((GOLD / "oracle" / "128x128.json").read_text())
    assert reynolds == pytest.approx(m["reynolds_last_av"], rel=1e-5)
    assert "MLUPS" in out


@pytest.mark.parametrize("opt", [["--tolerance"], ["--kernel", "stream"], ["--spl", "4"], ["-n", "4"],
                                 ["--graph-steps", "8"]])
def test_cpu_device_refuses_gpu_only_options(tmp_path, opt):
    """--device cpu has one numerics and one kernel: a '--device cpu --tolerance'
    run must fail loudly instead of writing bitwise results."""
    r = subprocess.run([str(EXE), "--device", "cpu", "--params", str(GOLD / "params" / "input_128x128.params"),
                        "--obstacles", str(GOLD / "params" / "obstacles_128x128.dat"), "--runs", "0",
                        "--out-dir", str(tmp_path)] + opt, capture_output=True, text=True, timeout=60)
    assert r.returncode != 0
    assert "GPU-only" in r.stderr and opt[0] in r.stderr
    assert not (tmp_path / "av_vels.dat").exists()
