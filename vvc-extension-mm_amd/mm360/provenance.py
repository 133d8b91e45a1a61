"""Build provenance of the HIP library: which sources the measured binary was compiled from.

__graft_entry__.build() recompiles lib/libmm360.so from the tree (make -B) and writes
lib/BUILD_INFO.json: the sha256 of the library it produced, of the sources it compiled and of the
compiler.  bench.py puts `provenance()` into its line, so the measured binary can be traced to the
committed sources (the hipcc build is deterministic: rebuilding the same sources gives the same sha).
"""
from __future__ import annotations

import glob
import hashlib
import json
import os
from typing import Optional

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROOT = os.path.dirname(PKG)
INFO_PATH = os.path.join(PKG, "lib", "BUILD_INFO.json")


def source_files():
    return sorted(glob.glob(os.path.join(PKG, "csrc", "*"))) + [os.path.join(ROOT, "include", "mm360.h"),
                                                                 os.path.join(PKG, "Makefile")]


def source_sha256() -> str:
    h = hashlib.sha256()
    for f in source_files():
        h.update(os.path.relpath(f, ROOT).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def file_sha256(path: str) -> str:
    with open(path, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()


def write_build_info(lib_path: str, compiler: str, command: str) -> dict:
    import datetime
    info = {"lib_sha256": file_sha256(lib_path), "src_sha256": source_sha256(),
            "sources": [os.path.relpath(f, ROOT) for f in source_files()], "compiler": compiler,
            "command": command, "built_utc": datetime.datetime.utcnow().strftime("%Y-%m-%dT%H:%M:%SZ")}
    with open(INFO_PATH, "w") as fh:
        json.dump(info, fh, indent=1)
    return info


def provenance(lib_path: str) -> dict:
    """The measured library against the record of its last build() and the tree's sources now."""
    out = {"lib_sha256": file_sha256(lib_path), "src_sha256": source_sha256()}
    info: Optional[dict] = None
    if os.path.exists(INFO_PATH):
        with open(INFO_PATH) as fh:
            info = json.load(fh)
    if info is None:
        out["build_info"] = "missing (library not built by __graft_entry__.build())"
        return out
    out["built_by_build"] = info.get("lib_sha256") == out["lib_sha256"]
    out["sources_unchanged_since_build"] = info.get("src_sha256") == out["src_sha256"]
    out["built_utc"] = info.get("built_utc")
    out["compiler"] = info.get("compiler")
    return out
