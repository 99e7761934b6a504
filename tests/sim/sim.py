"""ctypes driver of tests/sim/cglane_sim.cpp (TEST INFRASTRUCTURE): the fit kernel's optimizer state machine on
the CPU, answered by the CPU restatement (oracle/)."""
import ctypes
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

_lib = None
_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int32)


def lib():
    global _lib
    if _lib is None:
        O.lib()
        subprocess.check_call(["make", "-s", "-C", HERE])
        L = ctypes.CDLL(os.path.join(HERE, "_build", "libcglane_sim.so"))
        L.sim_fit_batch.argtypes = [_dp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_int, _dp, ctypes.c_int, ctypes.c_int, _dp, _dp, _ip, _ip]
        _lib = L
    return _lib


def sim_fit(series, p, d, q, I, smear=O.DEFAULT_SMEAR, ns=1, nc=1):
    """CG fits of `series` (N x T) from the Hannan-Rissanen init, by the kernel's state machine. Series whose HR
    init fails are skipped (status -1). Returns dict(status, coef, ll, n_eval, n_grad, passes_f, passes_g,
    spec_hits, chains)."""
    series = np.ascontiguousarray(np.atleast_2d(series), dtype=np.float64)
    N, T = series.shape
    k = p + q + I
    n = T - d
    y = np.stack([O.differences_of_order_d(s, d)[d:] for s in series]) if N else np.zeros((0, n))
    y = np.ascontiguousarray(y)
    init = np.zeros((N, k))
    ok = np.zeros(N, bool)
    for i in range(N):
        st, x0 = O.hannan_rissanen(y[i], p, q, I)
        if st == 0:
            init[i] = x0
            ok[i] = True
    coef = np.full((N, k), np.nan)
    ll = np.full(N, np.nan)
    status = np.full(N, -1, np.int32)
    counts = np.zeros((N, 14), np.int32)
    idx = np.nonzero(ok)[0]
    if len(idx):
        yy = np.ascontiguousarray(y[idx])
        ii = np.ascontiguousarray(init[idx])
        c = np.empty((len(idx), k))
        l = np.empty(len(idx))
        s = np.empty(len(idx), np.int32)
        cn = np.empty((len(idx), 14), np.int32)
        rc = lib().sim_fit_batch(yy.ctypes.data_as(_dp), len(idx), n, n, p, q, I, smear, ii.ctypes.data_as(_dp),
                                 ns, nc, c.ctypes.data_as(_dp), l.ctypes.data_as(_dp), s.ctypes.data_as(_ip),
                                 cn.ctypes.data_as(_ip))
        assert rc == 0, rc
        coef[idx], ll[idx], status[idx], counts[idx] = c, l, s, cn
    return dict(status=status, coef=coef, ll=ll, n_eval=counts[:, 0], n_grad=counts[:, 1], passes_f=counts[:, 2],
                passes_g=counts[:, 3], spec_hits=counts[:, 4], chains=counts[:, 5], f_by_phase=counts[:, 6:])


def nan_iter_evals(dir_finite=True):
    """Evaluations per CG iteration in the NaN-absorbing state, stepped (no fast-forward), and the kernel's constant."""
    L = lib()
    return L.sim_nan_iter_evals(int(dir_finite)), L.sim_k_nan_iter_evals()
