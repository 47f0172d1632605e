"""Adjacency / feature normalisation (host side, fp64) -- drop-in for the
reference's normalization.py.

The values of S decide the arithmetic of the whole hot path, so this module
reproduces the reference's numbers bit for bit (pinned by
tests/test_dropin.py::test_aug_normalized_adjacency_matches_reference against
the reference module itself, and on the device by tests/test_gpu_normalize.py
against the reference's S hashes):

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


def aug_normalize_on_device(adj, device="cuda"):
    """S = AugNorm(A) computed on the GPU (libsgc_amd: sgc_augnorm_count/fill),
    bit-identical to aug_normalized_adjacency(A) -> fp32.  Returns a
    sgc_amd.propagate.DeviceCSR ready for propagation.

    A must be canonical CSR (scipy's has_canonical_format: sorted, unique
    columns), which is what the loaders produce (networkx adjacency, A + A^T).
    The only host step is the one the reference itself does in numpy:
    d = rowsum ** -0.5 with inf -> 0 (normalization.py:8-10)."""
    return aug_normalize_device_arrays(*device_csr64(adj, device))


def device_csr64(adj, device="cuda"):
    """Canonical scipy CSR A -> (row_ptr int32, col_idx int32, val fp64, n)
    on the device: the input of the on-device AugNorm and sub-graph kernels."""
    import torch
    a = sp.csr_matrix(adj)
    if not a.has_canonical_format:
        raise ValueError("sgc_amd: A must be canonical CSR (sorted unique column indices); "
                         "use aug_normalized_adjacency")
    if a.shape[0] != a.shape[1]:
        raise ValueError("sgc_amd: A must be square")
    n = a.shape[0]
    if n >= 2**31 - 1 or a.nnz >= 2**31 - 1:
        raise ValueError("sgc_amd: beyond int32 CSR")
    dev = torch.device(device)
    rp = torch.from_numpy(a.indptr.astype(np.int32)).to(dev)
    ci = torch.from_numpy(a.indices.astype(np.int32)).to(dev)
    va = torch.from_numpy(a.data.astype(np.float64)).to(dev)
    return rp, ci, va, n


def subgraph_on_device(rp, ci, va, n, idx):
    """B = A[idx][:, idx] on the device (reference utils.py:117, the inductive
    train sub-graph), from device_csr64 arrays: canonical CSR with fp64 values
    (new row i = old row idx[i], new column = position in idx), ready for
    aug_normalize_device_arrays -- whose S is then the reference's
    fetch_normalization('AugNormAdj')(adj[idx, :][:, idx]) bit for bit.
    Repeated ids raise ValueError (the host slice handles them)."""
    import torch

    from . import _lib
    from .propagate import ctypes_byref
    dev = rp.device
    idx_t = torch.as_tensor(np.asarray(idx, dtype=np.int64)).to(dev)
    m, nnz = int(idx_t.numel()), int(ci.numel())
    lib = _lib.load()
    ws_bytes = lib.sgc_subgraph_workspace(n, m, nnz)
    ws = torch.empty(max(1, ws_bytes), dtype=torch.uint8, device=dev)
    out_rp = torch.empty(m + 1, dtype=torch.int32, device=dev)
    total, status = _lib._i64(0), _lib._u32(0)
    with torch.cuda.device(dev):
        stream = _lib.stream_handle(dev)
        rc = lib.sgc_subgraph_count(_lib.ptr(rp), _lib.ptr(ci), n, nnz, _lib.ptr(idx_t), m,
                                    _lib.ptr(out_rp), _lib.ptr(ws), ws_bytes, ctypes_byref(total),
                                    ctypes_byref(status), stream)
        if rc == 1 and status.value & 1:
            raise ValueError("subgraph_on_device: repeated indices")
        _lib.check(rc, "subgraph_count")
        t = int(total.value)
        out_ci = torch.empty(max(t, 1), dtype=torch.int32, device=dev)
        out_va = torch.empty(max(t, 1), dtype=torch.float64, device=dev)
        _lib.check(lib.sgc_subgraph_fill(_lib.ptr(rp), _lib.ptr(ci), _lib.ptr(va), n, nnz,
                                         _lib.ptr(idx_t), m, _lib.ptr(out_rp), _lib.ptr(out_ci),
                                         _lib.ptr(out_va), _lib.ptr(ws), ws_bytes, stream),
                   "subgraph_fill")
    return out_rp, out_ci[:t], out_va[:t], m


def aug_normalize_device_arrays(rp, ci, va, n):
    """S = AugNorm(A) on the device from canonical CSR arrays (device_csr64 /
    subgraph_on_device); see aug_normalize_on_device."""
    import torch

    from . import _lib
    from .propagate import DeviceCSR, ctypes_byref
    dev = rp.device
    a_nnz = int(ci.numel())
    lib = _lib.load()
    out_rp = torch.empty(n + 1, dtype=torch.int32, device=dev)
    rowsum = torch.empty(max(n, 1), dtype=torch.float64, device=dev)
    ws_bytes = lib.sgc_augnorm_workspace(n)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    nnz_out, status = _lib._i64(0), _lib._u32(0)
    with torch.cuda.device(dev):
        stream = _lib.stream_handle(dev)
        _lib.check(lib.sgc_augnorm_count(_lib.ptr(rp), _lib.ptr(ci), _lib.ptr(va), n, a_nnz,
                                         _lib.ptr(out_rp), _lib.ptr(rowsum), _lib.ptr(ws), ws_bytes,
                                         ctypes_byref(nnz_out), ctypes_byref(status), stream),
                   "augnorm_count")
        d = torch.from_numpy(_inv_power(rowsum[:n].cpu().numpy(), -0.5)).to(dev)
        total = int(nnz_out.value)
        out_ci = torch.empty(max(total, 1), dtype=torch.int32, device=dev)
        out_va = torch.empty(max(total, 1), dtype=torch.float32, device=dev)
        _lib.check(lib.sgc_augnorm_fill(_lib.ptr(rp), _lib.ptr(ci), _lib.ptr(va), n, _lib.ptr(d),
                                        _lib.ptr(out_rp), _lib.ptr(out_ci), _lib.ptr(out_va),
                                        _lib.ptr(ws), ws_bytes, ctypes_byref(nnz_out), stream),
                   "augnorm_fill")
    total = int(nnz_out.value)
    csr = DeviceCSR(n, n, out_rp, out_ci[:total], out_va[:total])
    csr.status = 1 | 2  # rows sorted, columns ascending (canonical A + I)
    return csr
