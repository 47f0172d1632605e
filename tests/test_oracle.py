"""The CPU oracle (oracle/spmm_oracle.c) against the reference's golden vectors.

The oracle is trusted as the checker only because these tests pin it: every
tiny case and every shape hash in tests/golden/ was produced by the
reference's own sgc_precompute (torch.spmm on CPU) in the build container.
"""
import hashlib
import os

import numpy as np
import pytest

from sgc_amd import graphs


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_oracle_tiny_cases_bit_exact(tiny_cases, oracle):
    for name, c in tiny_cases.items():
        n = int(c["n"])
        rp, ci, va = oracle.coo_to_csr(n, n, c["rows"], c["cols"], c["vals"])
        for key in sorted(k for k in c if k.startswith("Y")):
            K = int(key[1:])
            got = oracle.propagate(rp, ci, va, c["X"], K)
            assert np.array_equal(got.view(np.uint32), c[key].view(np.uint32)), (name, K)


def test_oracle_coo_storage_order_equals_stable_csr(tiny_cases, oracle):
    """Direct storage-order COO FMA == stable row sort + CSR (unsorted/dup input)."""
    c = tiny_cases["raw_unsorted_dups_F7"]
    n = int(c["n"])
    Y_coo = oracle.spmm_coo(n, c["rows"], c["cols"], c["vals"], c["X"])
    rp, ci, va = oracle.coo_to_csr(n, n, c["rows"], c["cols"], c["vals"])
    Y_csr = oracle.spmm_csr(rp, ci, va, c["X"])
    assert np.array_equal(Y_coo.view(np.uint32), Y_csr.view(np.uint32))
    assert np.array_equal(Y_coo.view(np.uint32), c["Y1"].view(np.uint32))


def test_oracle_row_slices(tiny_cases, oracle):
    c = tiny_cases["norm_n48_F65"]
    n = int(c["n"])
    rp, ci, va = oracle.coo_to_csr(n, n, c["rows"], c["cols"], c["vals"])
    full = oracle.spmm_csr(rp, ci, va, c["X"])
    parts = [oracle.spmm_csr(rp, ci, va, c["X"], a, b) for a, b in ((0, 7), (7, 30), (30, n))]
    assert np.array_equal(np.concatenate(parts), full)


def test_oracle_rejects_out_of_range(oracle):
    with pytest.raises(RuntimeError):
        oracle.coo_to_csr(3, 3, np.array([0, 3]), np.array([0, 1]), np.array([1.0, 2.0]))


@pytest.mark.parametrize("shape", ["cora", "pubmed"])
def test_oracle_shape_hashes(shape, shapes_golden, shape_rows, oracle):
    g = shapes_golden[shape]
    S = graphs.synthetic_graph(shape, seed=g["seed"])
    rows, cols, vals = S.coo()
    assert sha(np.stack([rows, cols])) == g["sha_indices"]
    assert sha(vals) == g["sha_values"]
    X = graphs.synthetic_features(shape, g["n"], g["features"], seed=g["feature_seed"])
    assert sha(X) == g["sha_X"]
    for K, rec in g["outputs"].items():
        Y = oracle.propagate(S.row_ptr, S.col_idx, S.val, X, int(K))
        pick = shape_rows[f"{shape}_rows"]
        assert np.array_equal(Y[pick], shape_rows[f"{shape}_K{K}"]), (shape, K)
        assert sha(Y) == rec["sha"], (shape, K)


def test_oracle_linear_matches_torch_fp32():
    import torch
    from oracle import oracle as o
    rng = np.random.default_rng(0)
    X = rng.standard_normal((300, 602)).astype(np.float32)
    W = rng.standard_normal((41, 602)).astype(np.float32) * 0.05
    b = rng.standard_normal(41).astype(np.float32)
    Y = o.linear(X, W, b)
    ref = torch.nn.functional.linear(torch.from_numpy(X), torch.from_numpy(W), torch.from_numpy(b))
    np.testing.assert_allclose(Y, ref.numpy(), rtol=1e-5, atol=1e-5)


def test_textsgc_oracle_matches_reference_golden(oracle):
    """The TextSGC restatement (oracle.textsgc_precompute) against the
    reference's own function's outputs (tests/golden/gen_textsgc.py)."""
    import scipy.sparse as sp
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "textsgc_case.npz"))
    n = int(z["n"])
    S = sp.csr_matrix((z["data"], z["indices"], z["indptr"]), shape=(n, n))
    coo = S.tocoo().astype(np.float32)
    rp, ci, va = oracle.coo_to_csr(n, n, coo.row, coo.col, coo.data)
    dense = np.asarray(S.todense()).astype(np.float32)
    idx = {k: z[f"idx_{k}"] for k in ("train", "val", "test")}
    got = oracle.textsgc_precompute(rp, ci, va, dense, idx)
    for k in ("train", "val", "test"):
        assert got[k].shape == z[f"feat_{k}"].shape, k
        assert np.array_equal(got[k].view(np.uint32), z[f"feat_{k}"].view(np.uint32)), k
