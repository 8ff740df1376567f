"""Hash of the HIP library's sources (csrc/*.hip, csrc/*.hpp, include/*.h).

The Makefile compiles it into liblbm_hip.so (lbm_source_hash()); the ctypes
binding recomputes it from the sources beside the library and refuses a
stale build.  Run as a script it prints the hash (the Makefile does that).
"""
from __future__ import annotations

import hashlib
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parent.parent   # lbm-graphcore_amd/
INCLUDE = PKG_ROOT.parent / "include"


def source_files():
    files = [("csrc/" + p.name, p) for p in (PKG_ROOT / "csrc").glob("*.hip")]
    files += [("csrc/" + p.name, p) for p in (PKG_ROOT / "csrc").glob("*.hpp")]
    files += [("include/" + p.name, p) for p in INCLUDE.glob("*.h")]
    return sorted(files)


def source_hash() -> str:
    h = hashlib.sha256()
    for name, path in source_files():
        h.update(name.encode() + b"\0")
        h.update(path.read_bytes())
        h.update(b"\0")
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(source_hash())
