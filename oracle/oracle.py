"""ctypes front-end for oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker.  The product path (sgc_amd) never does.

Restates /root/reference/utils.py:92-97 (sgc_precompute -> torch.spmm at
utils.py:95) as sequential fmaf chains in CSR order; see spmm_oracle.c.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


def build(force=False):
    if force or not os.path.exists(_LIB_PATH) or \
            os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "spmm_oracle.c")):
        subprocess.check_call(["make", "-s", "-C", _HERE, "liboracle.so"])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        i64, i32, p = ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p
        L.oracle_coo_to_csr.argtypes = [i64, i64, i64, p, p, p, p, p, p]
        L.oracle_spmm_csr.argtypes = [i64, i64, i64, p, p, p, p, i64, p, i64]
        L.oracle_spmm_coo.argtypes = [i64, i64, i64, p, p, p, p, i64, p, i64]
        L.oracle_propagate.argtypes = [i64, i64, i32, p, p, p, p, p, p]
        L.oracle_linear_f64acc.argtypes = [i64, i64, i64, p, p, p, p]
        for f in (L.oracle_coo_to_csr, L.oracle_spmm_csr, L.oracle_spmm_coo,
                  L.oracle_propagate, L.oracle_linear_f64acc):
            f.restype = ctypes.c_int
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"oracle {what} failed with code {rc}")


def coo_to_csr(n_rows, n_cols, rows, cols, vals):
    rows = np.ascontiguousarray(rows, dtype=np.int64)
    cols = np.ascontiguousarray(cols, dtype=np.int64)
    vals = np.ascontiguousarray(vals, dtype=np.float32)
    nnz = rows.shape[0]
    row_ptr = np.empty(n_rows + 1, np.int32)
    col_idx = np.empty(nnz, np.int32)
    val = np.empty(nnz, np.float32)
    _check(lib().oracle_coo_to_csr(n_rows, n_cols, nnz, _ptr(rows), _ptr(cols), _ptr(vals),
                                   _ptr(row_ptr), _ptr(col_idx), _ptr(val)), "coo_to_csr")
    return row_ptr, col_idx, val


def spmm_csr(row_ptr, col_idx, val, X, row_begin=0, row_end=None):
    X = np.ascontiguousarray(X, dtype=np.float32)
    n = row_ptr.shape[0] - 1
    row_end = n if row_end is None else row_end
    F = X.shape[1]
    Y = np.empty((row_end - row_begin, F), np.float32)
    _check(lib().oracle_spmm_csr(row_begin, row_end, F, _ptr(row_ptr), _ptr(col_idx), _ptr(val),
                                 _ptr(X), F, _ptr(Y), F), "spmm_csr")
    return Y


def spmm_coo(n_rows, rows, cols, vals, X):
    rows = np.ascontiguousarray(rows, dtype=np.int64)
    cols = np.ascontiguousarray(cols, dtype=np.int64)
    vals = np.ascontiguousarray(vals, dtype=np.float32)
    X = np.ascontiguousarray(X, dtype=np.float32)
    F = X.shape[1]
    Y = np.empty((n_rows, F), np.float32)
    _check(lib().oracle_spmm_coo(n_rows, rows.shape[0], F, _ptr(rows), _ptr(cols), _ptr(vals),
                                 _ptr(X), F, _ptr(Y), F), "spmm_coo")
    return Y


def propagate(row_ptr, col_idx, val, X0, K):
    X0 = np.ascontiguousarray(X0, dtype=np.float32)
    n, F = X0.shape
    out = np.empty_like(X0)
    work = np.empty_like(X0)
    _check(lib().oracle_propagate(n, F, K, _ptr(row_ptr), _ptr(col_idx), _ptr(val),
                                  _ptr(X0), _ptr(out), _ptr(work)), "propagate")
    return out


def linear(X, W, b):
    X = np.ascontiguousarray(X, dtype=np.float32)
    W = np.ascontiguousarray(W, dtype=np.float32)
    M, K = X.shape
    C = W.shape[0]
    Y = np.empty((M, C), np.float32)
    bp = _ptr(np.ascontiguousarray(b, dtype=np.float32)) if b is not None else None
    _check(lib().oracle_linear_f64acc(M, K, C, _ptr(X), _ptr(W), bp, _ptr(Y)), "linear")
    return Y


def textsgc_precompute(row_ptr, col_idx, val, dense, index_dict):
    """TextSGC's one-hop precompute restated (reference
    downstream/TextSGC/utils.py:131-152) on the oracle SpMM:
    for each split, F = (S . dense[:, idx])^T; train fixes the columns with a
    positive range over the training rows and their min/range; every split is
    (F[:, useful] - min) / range.  Returns {split: float32 array}."""
    import numpy as _np
    out = {}

    def hop(idx):
        X = _np.ascontiguousarray(dense[:, _np.asarray(idx)], dtype=_np.float32)
        return _np.ascontiguousarray(spmm_csr(row_ptr, col_idx, val, X).T)

    tr = hop(index_dict["train"])
    mx, mn = tr.max(axis=0, keepdims=True), tr.min(axis=0, keepdims=True)
    rng = mx - mn
    useful = _np.nonzero(rng.squeeze(0) > 0)[0]
    mn, rng = mn[:, useful], rng[:, useful]
    out["train"] = (tr[:, useful] - mn) / rng
    for phase in ("test", "val"):
        out[phase] = (hop(index_dict[phase])[:, useful] - mn) / rng
    return out
