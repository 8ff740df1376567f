"""bench.py's aux watchdog (CPU): a hanging aux measurement must not cost the
line -- past the budget rank 0 prints the line with the aux done so far and
every rank exits with bench.WATCHDOG_EXIT (3, so the launcher sees that an aux
hung); within the budget the line is printed exactly once and the exit is 0."""
from __future__ import annotations

import json
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]

PROLOG = "import sys, time; sys.path[:0] = [{root!r}, {pkg!r}]; import bench\n".format(
    root=str(ROOT), pkg=str(ROOT / "lbm-graphcore_amd"))


def run(code: str, timeout: float = 60):
    t0 = time.time()
    p = subprocess.run([sys.executable, "-c", PROLOG + code], capture_output=True, text=True, timeout=timeout)
    return p, time.time() - t0


def test_watchdog_prints_and_exits_on_hang():
    p, dt = run('out = {"metric": "m", "value": 1.0, "aux": {}}\n'
                'w = bench.AuxWatchdog(0.5, out, 0)\n'
                'out["aux"]["done_before_hang"] = 1\n'
                'time.sleep(30)\n'
                'print("not reached")\n')
    assert p.returncode == 3, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and "not reached" not in p.stdout
    d = json.loads(lines[0])
    assert d["value"] == 1.0 and d["aux"]["done_before_hang"] == 1 and "watchdog" in d["aux"]
    assert dt < 20


def test_watchdog_other_ranks_exit_silently():
    p, _ = run('out = {"metric": "m", "value": 1.0}\n'
               'w = bench.AuxWatchdog(0.5, out, 3)\n'
               'time.sleep(30)\n')
    assert p.returncode == 3 and p.stdout.strip() == ""


def test_watchdog_finish_prints_once():
    p, _ = run('out = {"metric": "m", "value": 2.0, "aux": {"x": 1}}\n'
               'w = bench.AuxWatchdog(5.0, out, 0)\n'
               'w.finish(); w.finish()\n')
    assert p.returncode == 0
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert lines == [json.dumps({"metric": "m", "value": 2.0, "aux": {"x": 1}})]


def test_main_watchdog_multi_rank_hang():
    """N > 1: a hung multi-rank check / timed measurement ends every rank with
    status 4; rank 0 prints a line naming the failure (no value)."""
    p, dt = run('w = bench.main_watchdog(0.5, 0, 8)\n'
                'time.sleep(30)\n')
    assert p.returncode == bench_exit("MAIN_WATCHDOG_EXIT") == 4, p.stderr
    d = json.loads(p.stdout.strip())
    assert d["value"] is None and d["n_gpus"] == 8 and "exceeded" in d["error"]
    assert dt < 20
    p, _ = run('w = bench.main_watchdog(0.5, 5, 8)\ntime.sleep(30)\n')
    assert p.returncode == 4 and p.stdout.strip() == ""


def test_main_watchdog_off_for_one_gpu_and_cancellable():
    p, _ = run('assert bench.main_watchdog(0.5, 0, 1) is None\n'
               'w = bench.main_watchdog(0.5, 0, 2); w.cancel(); time.sleep(1.0); print("ok")\n')
    assert p.returncode == 0 and p.stdout.strip() == "ok"


def bench_exit(name: str) -> int:
    sys.path[:0] = [str(ROOT), str(ROOT / "lbm-graphcore_amd")]
    import bench
    return getattr(bench, name)
