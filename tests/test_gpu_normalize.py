"""On-device AugNorm vs the reference's S, bit for bit.

The golden shape hashes (tests/golden/shapes.json) are of S exactly as the
reference builds it (normalization.py:5-12 + utils.py:23-30); the host
restatement sgc_amd.normalization.aug_normalized_adjacency is pinned to the
reference by tests/test_dropin.py and serves as the checker for the
randomised cases.
"""
import hashlib
import os
import sys

import numpy as np
import pytest
import scipy.sparse as sp
import torch

pytestmark = pytest.mark.gpu


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def csr_coo_host(csr):
    rp = csr.row_ptr.cpu().numpy().astype(np.int64)
    rows = np.repeat(np.arange(csr.n_rows, dtype=np.int64), np.diff(rp))
    return rows, csr.col_idx.cpu().numpy().astype(np.int64), csr.val.cpu().numpy()


def binary_sym(n, u, v):
    A = sp.coo_matrix((np.ones(len(u)), (u, v)), shape=(n, n)).tocsr()
    return A + A.T


@pytest.mark.parametrize("shape", ["cora", "pubmed", "reddit"])
def test_device_augnorm_matches_reference_hash(shape, shapes_golden):
    from sgc_amd import graphs
    from sgc_amd.normalization import aug_normalize_on_device
    g = shapes_golden[shape]
    u, v = graphs.rmat_pairs(g["n"], g["edges"], seed=g["seed"])
    csr = aug_normalize_on_device(binary_sym(g["n"], u, v))
    rows, cols, vals = csr_coo_host(csr)
    assert csr.nnz == g["nnz"]
    assert sha(np.stack([rows, cols])) == g["sha_indices"]
    assert sha(vals) == g["sha_values"]


def _cases():
    rng = np.random.default_rng(11)
    n = 400
    out = {}
    r, c = rng.integers(0, n, 3000), rng.integers(0, n, 3000)
    A = sp.coo_matrix((np.ones(3000), (r, c)), shape=(n, n)).tocsr()
    out["with_selfloops"] = A  # duplicates summed by tocsr -> weights >= 1
    B = sp.coo_matrix((rng.integers(1, 4, 3000).astype(float), (r, c)), shape=(n, n)).tocsr()
    out["weighted_sym"] = B + B.T
    C = sp.coo_matrix((rng.standard_normal(3000), (r, c)), shape=(n, n)).tocsr()
    out["real_weights"] = C
    D = sp.csr_matrix((n, n))
    out["empty"] = D
    E = sp.lil_matrix((6, 6))
    E[0, 0] = -1.0  # a_00 + 1 == 0 -> pruned; row 0 sums to 0 -> d_0 = 0
    E[0, 3] = 1.0
    E[1, 2] = 2.0
    E[2, 1] = 2.0
    out["zero_diag_row"] = E.tocsr()
    return out


@pytest.mark.parametrize("name", list(_cases()))
def test_device_augnorm_matches_host_restatement(name):
    from sgc_amd.normalization import aug_normalize_on_device, aug_normalized_adjacency
    A = _cases()[name]
    A.sum_duplicates()
    A.sort_indices()
    want = aug_normalized_adjacency(A)
    got = aug_normalize_on_device(A)
    rows, cols, vals = csr_coo_host(got)
    assert np.array_equal(rows, want.row) and np.array_equal(cols, want.col), name
    assert np.array_equal(vals.view(np.uint32), want.data.astype(np.float32).view(np.uint32)), name


def test_device_augnorm_rejects_noncanonical():
    from sgc_amd.normalization import aug_normalize_on_device
    A = sp.csr_matrix((np.ones(3), np.array([2, 1, 0]), np.array([0, 3, 3, 3])), shape=(3, 3))
    with pytest.raises(ValueError):
        aug_normalize_on_device(A)


def test_to_torch_coo_and_cached_propagation(tiny_cases, shapes_golden, shape_rows):
    """The loaders' adjacency tensor: reference COO layout + attached CSR."""
    from sgc_amd import graphs
    from sgc_amd.normalization import aug_normalize_on_device
    from sgc_amd.propagate import to_torch_coo
    from sgc_amd.utils import sgc_precompute
    g = shapes_golden["pubmed"]
    u, v = graphs.rmat_pairs(g["n"], g["edges"], seed=g["seed"])
    adj = to_torch_coo(aug_normalize_on_device(binary_sym(g["n"], u, v)))
    assert adj.is_sparse and not adj.is_coalesced() and adj.dtype == torch.float32
    idx = adj._indices().cpu().numpy()
    assert sha(idx) == g["sha_indices"]
    assert sha(adj._values().cpu().numpy()) == g["sha_values"]
    X = graphs.synthetic_features("pubmed", g["n"], g["features"], seed=g["feature_seed"])
    out, _ = sgc_precompute(torch.from_numpy(X).cuda(), adj, 2)
    assert sha(out.cpu().numpy()) == g["outputs"]["2"]["sha"]


def test_load_citation_device_equals_host(tmp_path, monkeypatch):
    sys.path.insert(0, os.path.dirname(__file__))
    from test_dropin import _write_planetoid
    from sgc_amd.utils import load_citation
    _write_planetoid(str(tmp_path), "citeseer", np.random.default_rng(3), isolated=True)
    monkeypatch.chdir(tmp_path)
    a = load_citation("citeseer", "AugNormAdj", cuda=False)
    b = load_citation("citeseer", "AugNormAdj", cuda=True)
    assert torch.equal(a[0]._indices(), b[0]._indices().cpu())
    assert torch.equal(a[0]._values(), b[0]._values().cpu())
    for x, y in zip(a[1:], b[1:]):
        assert torch.equal(x, y.cpu())


# ---------------------------------------------------------------------------
# Induced sub-graph A[idx][:, idx] on the device.

def _sub_host(A, idx):
    """The reference's slice (utils.py:117), canonicalised."""
    B = sp.csr_matrix(A[idx, :][:, idx])
    B.sum_duplicates()
    B.sort_indices()
    return B


@pytest.mark.parametrize("order", ["ascending", "shuffled", "empty", "all", "single"])
def test_device_subgraph_matches_scipy_slice(order):
    from sgc_amd.normalization import device_csr64, subgraph_on_device
    rng = np.random.default_rng(5)
    A = _cases()["weighted_sym"]
    A.sum_duplicates()
    A.sort_indices()
    n = A.shape[0]
    idx = {"ascending": np.sort(rng.choice(n, 250, replace=False)),
           "shuffled": rng.choice(n, 250, replace=False),
           "empty": np.zeros(0, np.int64), "all": rng.permutation(n),
           "single": np.array([7])}[order]
    rp, ci, va, m = subgraph_on_device(*device_csr64(A), idx)
    want = _sub_host(A, idx)
    assert m == len(idx)
    assert np.array_equal(rp.cpu().numpy(), want.indptr)
    assert np.array_equal(ci.cpu().numpy(), want.indices)
    assert np.array_equal(va.cpu().numpy().view(np.uint64), want.data.view(np.uint64))


def test_device_subgraph_rejects_bad_ids():
    from sgc_amd.normalization import device_csr64, subgraph_on_device
    A = _cases()["weighted_sym"]
    A.sum_duplicates()
    A.sort_indices()
    with pytest.raises(ValueError):
        subgraph_on_device(*device_csr64(A), np.array([3, 5, 3]))
    with pytest.raises(RuntimeError):
        subgraph_on_device(*device_csr64(A), np.array([3, 400]))


@pytest.mark.slow
def test_device_inductive_s_train_reddit_shape(shapes_golden):
    """Reddit-shape A + A^T, a shuffled 65% train index: S_train from the
    device slice + device AugNorm equals the reference recipe on the host
    (slice, then normalization.py:5-12), bit for bit."""
    from sgc_amd import graphs
    from sgc_amd.normalization import (aug_normalize_device_arrays, aug_normalized_adjacency,
                                       device_csr64, subgraph_on_device)
    g = shapes_golden["reddit"]
    u, v = graphs.rmat_pairs(g["n"], g["edges"], seed=g["seed"])
    A = binary_sym(g["n"], u, v)
    rng = np.random.default_rng(1)
    idx = rng.choice(g["n"], int(0.65 * g["n"]), replace=False)
    got = aug_normalize_device_arrays(*subgraph_on_device(*device_csr64(A), idx))
    want = aug_normalized_adjacency(A[idx, :][:, idx])
    rows, cols, vals = csr_coo_host(got)
    assert np.array_equal(rows, want.row) and np.array_equal(cols, want.col)
    assert np.array_equal(vals.view(np.uint32), want.data.astype(np.float32).view(np.uint32))


def test_load_reddit_device_equals_host(tmp_path, monkeypatch):
    """load_reddit_data (utils.py:110-131) on the device path vs the host
    path on a small npz pair written here: adj, train_adj, features, labels."""
    from sgc_amd.utils import load_reddit_data
    rng = np.random.default_rng(4)
    n = 300
    r, c = rng.integers(0, n, 2000), rng.integers(0, n, 2000)
    A = sp.coo_matrix((np.ones(2000), (r, c)), shape=(n, n)).tocsr()
    A.data[:] = 1.0
    data = tmp_path / "data"
    data.mkdir()
    sp.save_npz(str(data / "reddit_adj.npz"), A)
    perm = rng.permutation(n)
    tr, va, te = np.sort(perm[:180]), np.sort(perm[180:240]), np.sort(perm[240:])
    np.savez(str(data / "reddit.npz"), feats=rng.standard_normal((n, 12)).astype(np.float32),
             y_train=rng.integers(0, 5, 180), y_val=rng.integers(0, 5, 60),
             y_test=rng.integers(0, 5, 60), train_index=tr, val_index=va, test_index=te)
    monkeypatch.chdir(tmp_path)
    a = load_reddit_data("AugNormAdj", "AugNormAdj", cuda=False)
    b = load_reddit_data("AugNormAdj", "AugNormAdj", cuda=True)
    for x, y in zip(a[:2], b[:2]):
        assert torch.equal(x._indices(), y._indices().cpu())
        assert torch.equal(x._values(), y._values().cpu())
    assert torch.equal(a[2], b[2].cpu()) and torch.equal(a[3], b[3].cpu())
