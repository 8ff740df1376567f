"""Host code under ASan + UBSan (SURVEY §5 sanitizer row; CPU only).

tests/sanitize/host_check.cpp drives the host loaders / writers
(lbm-graphcore_amd/host/lbm_host.hpp) and the CPU oracle with
-fsanitize=address,undefined -fno-sanitize-recover=all: any out-of-bounds
access, use-after-free, leak or undefined behaviour aborts the run.  The
device side has its own read-before-write check (LBM_POISON,
tests/test_poison.py); GPU sanitizers are not available on this pool."""
from __future__ import annotations

import shutil
import subprocess

import pytest

from conftest import GOLD, ROOT

SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_code_under_asan_ubsan(tmp_path):
    build = tmp_path / "build"
    build.mkdir()
    objs = []
    for src in ("lbm_oracle.c", "lbm_oracle3d.c"):
        obj = build / (src + ".o")
        subprocess.run(["gcc", "-std=c11", "-ffp-contract=off", "-fopenmp", *SAN, "-c", str(ROOT / "oracle" / src),
                        "-o", str(obj)], check=True)
        objs.append(str(obj))
    exe = build / "host_check"
    subprocess.run(["g++", "-std=c++17", "-fopenmp", *SAN, "-I", str(ROOT / "include"),
                    str(ROOT / "tests" / "sanitize" / "host_check.cpp"), *objs, "-o", str(exe), "-lm"], check=True)
    work = tmp_path / "run"
    work.mkdir()
    r = subprocess.run([str(exe), str(GOLD / "params"), str(work)], capture_output=True, text=True, timeout=300,
                       env={"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0", "UBSAN_OPTIONS": "print_stacktrace=1",
                            "OMP_NUM_THREADS": "4", "PATH": "/usr/bin:/bin"})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr
    assert "host_check: ok" in r.stdout
    assert (work / "final_state.dat").stat().st_size > 0
