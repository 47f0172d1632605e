"""Adjacency / feature normalisation (host side, fp64) -- drop-in for the
reference's normalization.py.

The values of S decide the arithmetic of the whole hot path, so this module
reproduces the reference's numbers bit for bit (pinned by
tests/test_normalization.py against fixtures made with the reference):

* aug_normalized_adjacency (reference normalization.py:5-12):
  S = D^-1/2 (A + I) D^-1/2 with D = rowsum(A + I), all in fp64;
  d = rowsum ** -0.5 via np.power, inf -> 0; entry = (d_i * a_ij) * d_j;
  entries in canonical CSR order (row-major, ascending column).
* row_normalize (reference normalization.py:21-28): X <- diag(1/rowsum) X,
  inf -> 0.
* fetch_normalization (reference normalization.py:14-19): only 'AugNormAdj'
  exists; any other name yields a zero-argument callable, so calling it with
  the adjacency raises TypeError exactly as the reference does.
"""
import numpy as np
import scipy.sparse as sp


def _inv_power(v, p):
    with np.errstate(divide="ignore"):
        out = np.power(v, p)
    out[np.isinf(out)] = 0.0
    return out


def aug_normalized_adjacency(adj):
    a = sp.csr_matrix(adj + sp.eye(adj.shape[0]))
    a.sum_duplicates()
    a.sort_indices()
    rowsum = np.asarray(a.sum(axis=1), dtype=np.float64).ravel()
    d = _inv_power(rowsum, -0.5)
    rows = np.repeat(np.arange(a.shape[0]), np.diff(a.indptr))
    data = (d[rows] * a.data.astype(np.float64)) * d[a.indices]
    return sp.coo_matrix((data, (rows, a.indices.copy())), shape=a.shape)


_NORMALIZERS = {"AugNormAdj": aug_normalized_adjacency}


def fetch_normalization(type):  # noqa: A002  (reference argument name)
    if type in _NORMALIZERS:
        return _NORMALIZERS[type]
    return lambda: "Invalid normalization technique."


def row_normalize(mx):
    # keep the row sums' dtype (float32 features stay float32, as the reference's)
    r_inv = _inv_power(np.asarray(mx.sum(1)).ravel(), -1)
    return sp.diags(r_inv).dot(mx)
