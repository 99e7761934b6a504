"""Build identity of libsparkts_arima.so, used to tie carried rocprofv3 PMC records to the build they measured.

hipcc's output is not byte-reproducible (two compiles of the same source differ in the offload bundle), so a
library rebuilt from unchanged sources gets a new sha256. Records therefore carry two keys: `build_sha` (the
profiled library itself) and `source_sha` (every input of the build: the HIP/C++ sources, the public header and
the Makefile with its compiler flags). A reader prefers the library match and says which key matched.
"""
import hashlib
import os

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB_PATH = os.path.join(PKG, "libsparkts_arima.so")


def library_sha(path=None):
    """sha256 of the library file (the one SPARKTS_ARIMA_LIB names, else the in-tree build); None if absent."""
    h = hashlib.sha256()
    try:
        with open(path or os.environ.get("SPARKTS_ARIMA_LIB", LIB_PATH), "rb") as f:
            for blk in iter(lambda: f.read(1 << 22), b""):
                h.update(blk)
    except OSError:
        return None
    return h.hexdigest()


def source_sha():
    """sha256 over the build's inputs, in a fixed order (file name + contents)."""
    files = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".hpp", ".cpp")) or f == "Makefile")
    paths = [os.path.join(CSRC, f) for f in files] + [os.path.join(ROOT, "include", "sparkts_arima.h")]
    h = hashlib.sha256()
    for p in paths:
        h.update(os.path.relpath(p, ROOT).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()


def match_record(recs, workload, lib_sha, src_sha):
    """The record of `workload` for this build: library sha first, then source sha. Returns (record, key) or
    (None, None)."""
    for key, val in (("build_sha", lib_sha), ("source_sha", src_sha)):
        if val is None:
            continue
        for m in recs:
            if m.get("workload") == workload and m.get(key) == val:
                return m, key
    return None, None
