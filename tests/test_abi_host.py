"""CPU-only checks of the C-ABI library and the host side (no compute calls).

* liblbm_hip.so loads and exports every function include/lbm_hip.h declares.
* Host-only ABI helpers: partition rule (StructuredGridUtils.hpp:472-561) and
  the halo plan.
* Without a GPU every compute entry point fails loudly (no CPU fallback).
* Problem I/O mirrors LbmParams.hpp / LatticeBoltzmannUtils.hpp; the check.py
  restatement behaves like the reference gate.
"""
from __future__ import annotations

import re
import subprocess

import numpy as np
import pytest

from conftest import GOLD, PKG, ROOT, load_problem
from lbm_amd import check as lcheck
from lbm_amd import io as lio
from lbm_amd import native


def header_symbols(name="lbm_hip.h", prefix="lbm_"):
    text = (ROOT / "include" / name).read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(rf"\b({prefix}[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_d3q19_symbol():
    L = native.load_library()
    syms = header_symbols("lbm3d_hip.h", "lbm3d_")
    assert len(syms) == 11
    assert sorted(native.EXPORTED3D) == syms
    out = subprocess.run(["nm", "-D", "--defined-only", str(native.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    for s in syms:
        assert hasattr(L, s), s
        assert re.search(rf"\bT {s}\b", out), s


def test_library_exports_every_declared_symbol():
    L = native.load_library()
    syms = header_symbols()
    assert len(syms) >= 17
    for s in syms:
        assert hasattr(L, s), s
    assert sorted(native.EXPORTED) == syms
    out = subprocess.run(["nm", "-D", "--defined-only", str(native.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    for s in syms:
        assert re.search(rf"\bT {s}\b", out), s
    assert L.lbm_abi_version() == 5


def test_stale_library_is_refused(monkeypatch):
    """The binding compares the library's compiled-in source hash with the
    sources beside it and refuses a stale build (no silent old kernels)."""
    from lbm_amd import srchash
    L = native.load_library()
    assert L.lbm_source_hash().decode() == srchash.source_hash()
    monkeypatch.setattr(native, "_lib", None)
    monkeypatch.setattr(srchash, "source_hash", lambda: "0000000000000000")
    with pytest.raises(RuntimeError, match="built from other sources"):
        native.load_library()


def test_no_torch_types_in_abi():
    text = (ROOT / "include" / "lbm_hip.h").read_text()
    assert "torch" not in text.lower().replace("torch.distributed", "")
    assert "hip_runtime" not in text  # plain C types only


def ref_partition(nx, ny, parts):
    """Python restatement of partitionForIpus (StructuredGridUtils.hpp:472-561)."""
    row_imb = np.float32(ny % parts) / np.float32(ny)
    col_imb = np.float32(nx % parts) / np.float32(nx)
    R = C = 1
    if parts == 2:
        R, C = (2, 1) if row_imb < col_imb else (1, 2)
    if parts == 4:
        R, C = 2, 2
    if parts == 8:
        R, C = (4, 2) if row_imb < col_imb else (2, 4)
    if parts == 16:
        R, C = 4, 4

    def rr(n, k):
        v = [0] * min(k, n)
        for i in range(n):
            v[i % len(v)] += 1
        return v

    if R > ny or C > nx:
        return R, C, None
    ra, ca = rr(ny, R), rr(nx, C)
    rects = {}
    y0 = 0
    for r, h in enumerate(ra):
        x0 = 0
        for c, w in enumerate(ca):
            rects[r * C + c] = (x0, y0, w, h)
            x0 += w
        y0 += h
    return R, C, [rects[i] for i in range(R * C)]


@pytest.mark.parametrize("nx,ny", [(128, 128), (128, 256), (256, 128), (1024, 1024), (37, 29), (16384, 16384),
                                   (8192, 16384), (100, 3)])
@pytest.mark.parametrize("parts", [1, 2, 4, 8, 16])
def test_partition_rule(nx, ny, parts):
    Rr, Cr, ref_rects = ref_partition(nx, ny, parts)
    if Rr > ny or Cr > nx:  # the reference would silently drop parts; we refuse
        with pytest.raises(native.LbmError):
            native.partition(nx, ny, parts)
        return
    R, C, rects = native.partition(nx, ny, parts)
    assert (R, C, rects) == (Rr, Cr, ref_rects)
    cover = np.zeros((ny, nx), np.int32)
    for x0, y0, w, h in rects:
        cover[y0:y0 + h, x0:x0 + w] += 1
    assert np.all(cover == 1)


def test_partition_explicit_grid_and_errors():
    R, C, rects = native.partition(128, 256, 6, 3, 2)
    assert (R, C) == (3, 2) and rects[0] == (0, 0, 64, 86) and rects[5] == (64, 171, 64, 85)
    for bad in [(128, 128, 3, 0, 0), (128, 128, 4, 3, 2), (4, 4, 8, 1, 8), (0, 4, 1, 0, 0)]:
        with pytest.raises(native.LbmError):
            native.partition(*bad)


def test_halo_plan():
    plan = native.halo_plan()
    cx = [0, 1, 0, -1, 0, 1, -1, -1, 1]
    cy = [0, 0, 1, 0, -1, 1, 1, -1, -1]
    assert [(dx, dy) for dx, dy, _ in plan] == [(cx[k], cy[k]) for k in range(1, 9)]
    for dx, dy, planes in plan:
        # exactly the speeds whose velocity has d's non-zero components
        want = [k for k in range(1, 9) if (dx == 0 or cx[k] == dx) and (dy == 0 or cy[k] == dy)]
        assert sorted(planes) == want


def test_compute_calls_fail_loudly_without_gpu():
    if native.device_count() > 0:
        pytest.skip("a GPU is visible; this checks the CPU-only container")
    p = lio.Params(16, 8, 4, 10, 0.1, 0.005, 1.85)
    with pytest.raises(native.LbmError) as ei:
        native.Engine(p, np.zeros((8, 16), np.uint8))
    assert ei.value.code == native.LBM_E_HIP


def test_runner_cli_errors():
    exe = PKG / "build" / "lbm_runner"
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode != 0 and "--params" in r.stderr
    r = subprocess.run([str(exe), "--params", "/nonexistent", "--obstacles", "/nonexistent"], capture_output=True,
                       text=True)
    assert r.returncode != 0 and "Could not parse parameters file" in r.stderr
    r = subprocess.run([str(PKG / "build" / "compare_lbm")], capture_output=True, text=True)
    assert r.returncode != 0 and "Usage" in r.stderr
    r = subprocess.run([str(exe), "--params", "p", "--obstacles", "o", "--kernel", "bogus"], capture_output=True,
                       text=True)
    assert r.returncode != 0 and "--kernel" in r.stderr


# ---------------------------------------------------------------- I/O ----

def test_params_loader():
    p = lio.Params.from_file(str(GOLD / "params" / "input_1024x1024.params"))
    assert (p.nx, p.ny, p.max_iters, p.reynolds_dim) == (1024, 1024, 20000, 10)
    assert p.density == np.float32(0.1) and p.accel == np.float32(0.01) and p.omega == np.float32(1.85)
    assert lio.Params.from_file("/nonexistent") is None


def test_obstacles_loader(tmp_path):
    p, obst = load_problem("1024x1024")
    assert obst.shape == (1024, 1024) and obst.dtype == np.uint8
    assert obst[:, 341].all() and obst[0].all() and obst[-1].all() and not obst[5, 5]
    assert int((obst == 0).sum()) == 1043462
    bad = tmp_path / "bad.dat"
    bad.write_text("1 1 1\n2 2 0\n")
    assert lio.read_obstacles(4, 4, str(bad)) is None
    bad.write_text("9 1 1\n")
    assert lio.read_obstacles(4, 4, str(bad)) is None


def test_writers_format(tmp_path):
    p = lio.Params(3, 2, 2, 10, 0.1, 0.005, 1.85)
    obst = np.array([[1, 0, 0], [0, 0, 0]], np.uint8)
    cells = lio.init_cells(p)
    cells[1, 2, 1] += 0.01
    lio.write_average_velocities(str(tmp_path / "a.dat"), np.array([1.5e-5, 2.0], np.float32))
    assert (tmp_path / "a.dat").read_text() == "0:\t1.499999962107e-05\n1:\t2.000000000000e+00\n"  # = C++ iostream output
    lio.write_results(str(tmp_path / "f.dat"), p, obst, cells)
    lines = (tmp_path / "f.dat").read_text().splitlines()
    assert len(lines) == 6
    assert lines[0] == "0 0 0.000000000000e+00 0.000000000000e+00 0.000000000000e+00 3.333333507180e-02 1"
    cols = lines[5].split()
    assert cols[:2] == ["2", "1"] and cols[6] == "0" and float(cols[2]) > 0


def test_check_restatement(tmp_path):
    ref_av = GOLD / "check" / "128x128.av_vels.dat.gz"
    ref_fs = GOLD / "check" / "128x128.final_state.dat.gz"
    assert lcheck.compare(ref_av, ref_fs, ref_av, ref_fs)["passed"]
    av = lcheck.load_av_vels(ref_av)
    fs = lcheck.load_final_state(ref_fs)
    av2 = av.copy()
    av2[100] *= 1.02
    res = lcheck.compare(av, fs, av2, fs)
    assert not res["passed"] and res["av"]["max_diff_step"] == 100
    fs2 = fs.copy()
    fs2[7, 2] *= 0.98
    assert not lcheck.compare(av, fs, av, fs2)["passed"]
    fs3 = fs.copy()
    fs3[3, 0] += 1
    assert lcheck.compare(av, fs, av, fs3)["reason"].startswith("Final state files coordinates")
    assert not lcheck.compare(av, fs, av[:-1], fs)["passed"]
    av4 = av.copy()
    av4[5] = np.nan
    assert not lcheck.compare(av, fs, av4, fs)["passed"]
    # CLI exit codes
    import gzip
    (tmp_path / "a.dat").write_bytes(gzip.decompress(ref_av.read_bytes()))
    (tmp_path / "f.dat").write_bytes(gzip.decompress(ref_fs.read_bytes()))
    args = ["--ref-av-vels-file", str(tmp_path / "a.dat"), "--ref-final-state-file", str(tmp_path / "f.dat"),
            "--av-vels-file", str(tmp_path / "a.dat"), "--final-state-file", str(tmp_path / "f.dat")]
    assert lcheck.main(args) == 0


def test_runner_partition_dump(tmp_path):
    import json
    exe = PKG / "build" / "lbm_runner"
    out = tmp_path / "partitioning.json"
    subprocess.run([str(exe), "--params", str(GOLD / "params" / "input_128x256.params"), "--obstacles",
                    str(GOLD / "params" / "obstacles_128x256.dat"), "-n", "8", "--dump-partitioning", str(out)],
                   capture_output=True, text=True)
    d = json.loads(out.read_text())["GridPartitioning"]
    assert len(d) == 8
    _, _, rects = native.partition(128, 256, 8)
    for i, e in enumerate(d):
        x0, y0, w, h = rects[i]
        assert e["ipu"] == i and e["slice"]["rows"] == {"from": y0, "to": y0 + h}
        assert e["slice"]["cols"] == {"from": x0, "to": x0 + w}
