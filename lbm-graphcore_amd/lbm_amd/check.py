"""Python 3 restatement of the reference gate check/check.py (Python 2 only).

Same CLI (``--ref-av-vels-file --ref-final-state-file --av-vels-file
--final-state-file [--tolerance 1]``, check.py:17-57), same arithmetic
(check.py:62-147): av_vels column 1 and final_state columns 0,1,5 are
loaded with numpy; coordinates must match exactly; step counts must match;
diff = ref - sim, pct = 100 * diff / (ref - diff); the run fails when the
worst |pct| exceeds the tolerance or is not finite.  Exit code 0 = pass.

``compare`` is the same check as a function for tests (it also accepts
arrays so fixtures need not be re-serialised).
"""
from __future__ import annotations

import argparse
import gzip
import sys

import numpy as np


def _open(path):
    return gzip.open(path, "rt") if str(path).endswith(".gz") else open(path, "r")


def load_av_vels(path) -> np.ndarray:
    with _open(path) as f:
        return np.loadtxt(f, usecols=[1], converters={1: lambda s: float(s)})


def load_final_state(path) -> np.ndarray:
    with _open(path) as f:
        return np.loadtxt(f, usecols=[0, 1, 5])


def diff_values(ref_vals: np.ndarray, sim_vals: np.ndarray) -> dict:
    diff = ref_vals - sim_vals
    with np.errstate(divide="ignore", invalid="ignore"):
        pct = 100.0 * (diff / (ref_vals - diff))
    step = int(np.argmax(np.abs(pct)))
    return {
        "max_diff_step": step,
        "max_diff": float(diff[step]),
        "max_diff_pcnt": float(pct[step]),
        "sim_val": float(sim_vals[step]),
        "ref_val": float(ref_vals[step]),
        "total": float(np.sum(np.abs(diff))),
    }


def compare(ref_av, ref_fs, sim_av, sim_fs, tolerance: float = 1.0, verbose: bool = False) -> dict:
    """Arrays or paths. Returns {'passed', 'av', 'fs', 'reason'}."""
    ref_av = load_av_vels(ref_av) if not isinstance(ref_av, np.ndarray) else ref_av
    sim_av = load_av_vels(sim_av) if not isinstance(sim_av, np.ndarray) else sim_av
    ref_fs = load_final_state(ref_fs) if not isinstance(ref_fs, np.ndarray) else ref_fs
    sim_fs = load_final_state(sim_fs) if not isinstance(sim_fs, np.ndarray) else sim_fs
    if ref_fs.shape != sim_fs.shape or np.any(ref_fs[:, 0:2] != sim_fs[:, 0:2]):
        return {"passed": False, "reason": "Final state files coordinates were not the same"}
    if ref_av.size != sim_av.size:
        return {"passed": False, "reason": "Different number of steps in av_vels files"}
    av = diff_values(ref_av, sim_av)
    fs = diff_values(ref_fs[:, 2], sim_fs[:, 2])
    loc = fs["max_diff_step"]
    fs["jj"] = int(sim_fs[loc, 0])
    fs["ii"] = int(sim_fs[loc, 1])
    fs_failed = (not np.isfinite(fs["max_diff_pcnt"])) or abs(fs["max_diff_pcnt"]) > tolerance
    av_failed = (not np.isfinite(av["max_diff_pcnt"])) or abs(av["max_diff_pcnt"]) > tolerance
    out = {"passed": not (fs_failed or av_failed), "av": av, "fs": fs, "av_failed": av_failed,
           "fs_failed": fs_failed, "reason": ""}
    if verbose:
        fmt = "  {sim_val:.12E} vs. {ref_val:.12E} = {max_diff_pcnt:.2g}%"
        print("Total difference in av_vels : {total:.12E}".format(**av))
        print("Biggest difference (at step {max_diff_step:d}) : {max_diff:.12E}".format(**av))
        print(fmt.format(**av))
        print()
        print("Total difference in final_state : {total:.12E}".format(**fs))
        print("Biggest difference (at coord ({jj:d},{ii:d})) : {max_diff:.12E}".format(**fs))
        print(fmt.format(**fs))
        print()
        if fs_failed:
            print("final state failed check")
        if av_failed:
            print("av_vels failed check")
        if out["passed"]:
            print("Both tests passed!")
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Testing script for HPC LBM coursework", fromfile_prefix_chars="@",
                                 formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    ap.add_argument("--tolerance", nargs=1, default=[1], type=float,
                    help="Percentage tolerance to match against reference results")
    ap.add_argument("--ref-av-vels-file", nargs=1, required=True, help="reference av_vels results file")
    ap.add_argument("--ref-final-state-file", nargs=1, required=True, help="reference final_state results file")
    ap.add_argument("--av-vels-file", nargs=1, required=True, help="calculated av_vels results file")
    ap.add_argument("--final-state-file", nargs=1, required=True, help="calculated final_state results file")
    a = ap.parse_args(argv)
    res = compare(a.ref_av_vels_file[0], a.ref_final_state_file[0], a.av_vels_file[0], a.final_state_file[0],
                  a.tolerance[0], verbose=True)
    if res.get("reason"):
        print(res["reason"])
    return 0 if res["passed"] else 1


if __name__ == "__main__":
    sys.exit(main())
