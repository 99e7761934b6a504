"""The C-ABI library loads and exports every symbol include/sparkts_arima.h declares (no GPU needed)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "sparkts_arima.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(arima_[a-z_]+)\s*\(", txt)))


def test_header_and_binding_agree():
    import sparkts_amd._lib as L
    assert declared_functions() == sorted(L.EXPORTED)


def test_library_exports_every_declared_symbol():
    import sparkts_amd._lib as L
    lib = L.load()
    nm = subprocess.check_output(["nm", "-D", "--defined-only", L.LIB_PATH], text=True)
    exported = set(re.findall(r" T (arima_\w+)", nm))
    for name in declared_functions():
        assert name in exported, name
        assert hasattr(lib, name)


def test_exports_are_plain_c_no_torch():
    import sparkts_amd._lib as L
    # the library's own NEEDED entries (not where the loader happens to resolve them: libamdhip64 may resolve into
    # a torch wheel's lib directory when one is on the search path)
    dyn = subprocess.check_output(["readelf", "-d", L.LIB_PATH], text=True)
    needed = [ln.split("[", 1)[1].split("]", 1)[0] for ln in dyn.splitlines() if "(NEEDED)" in ln]
    assert needed and not any("torch" in n or "c10" in n for n in needed), needed


def test_pure_host_entry_points():
    import sparkts_amd._lib as L
    lib = L.load()
    assert lib.arima_num_params(2, 2, 1) == 5 and lib.arima_num_params(0, 0, 0) == 0
    names = [lib.arima_status_name(i).decode() for i in range(16)]
    assert names == ["OK", "MAX_EVAL", "BRACKET_MAX_EVAL", "MAX_ITER", "SINGULAR", "NOT_ENOUGH_DATA", "NO_DATA",
                     "BAD_INTERVAL", "ZERO_PARAMS", "UNSUPPORTED_METHOD", "SERIES_TOO_SHORT", "NOT_STATIONARY",
                     "NO_MODEL", "UNKNOWN", "TOO_FEW_PARAMS", "UNKNOWN"]    # 13, 15 retired with RESCUE restated


def test_status_codes_match_oracle_numbering():
    import oracle as O
    import sparkts_amd._lib as L
    lib = L.load()
    for code, name in O.ST_NAMES.items():
        assert lib.arima_status_name(code).decode() == name


def test_product_path_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    import sparkts_amd._lib as L
    from sparkts_amd.models import ARIMA
    with pytest.raises(L.EngineError):
        ARIMA.fit_model(1, 0, 1, [1.0, 2.0, 3.0, 5.0, 4.0, 6.0, 5.0, 7.0])


def test_stats_struct_matches_binding():
    # arima_fit_stats (include/sparkts_arima.h) and the ctypes mirror (sparkts_amd._lib.FitStats): same fields, same
    # order, same types -- arima_get_last_stats writes the C layout into the Python structure
    import sparkts_amd._lib as L
    txt = open(HEADER).read()
    body = txt[txt.index("typedef struct arima_fit_stats {"):txt.index("} arima_fit_stats;")]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    fields = re.findall(r"\b(int64_t|double|int32_t)\s+(\w+)\s*(?:\[(\d+)\])?\s*;", body)
    ctypes_of = {"int64_t": ctypes.c_int64, "double": ctypes.c_double, "int32_t": ctypes.c_int32}
    want = [(n, ctypes_of[t] * int(k) if k else ctypes_of[t]) for t, n, k in fields]
    got = list(L.FitStats._fields_)
    assert [n for n, _ in want] == [n for n, _ in got]
    for (n, a), (_, b) in zip(want, got):
        assert ctypes.sizeof(a) == ctypes.sizeof(b) and getattr(a, "_type_", a) == getattr(b, "_type_", b), n
