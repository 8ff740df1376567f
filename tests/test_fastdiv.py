"""CPU evidence for the exact division sequences of the two-column stream
kernel (tools/check_fastdiv.c, header of lbm-graphcore_amd/csrc/lbm_stream2.hip):
constant divisors exhaustively over 41 binades, the variable-divisor sequence
on random (momentum, density) pairs with every 1-ulp reciprocal candidate."""
from __future__ import annotations

import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_fast_division_sequences_exact(tmp_path):
    exe = tmp_path / "check_fastdiv"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-mfma", str(ROOT / "tools" / "check_fastdiv.c"), "-lm",
                    "-o", str(exe)], check=True)
    r = subprocess.run([str(exe), "20000000"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "constant divisors: 0 mismatches" in r.stdout
    assert "variable divisor: 0 mismatches" in r.stdout
