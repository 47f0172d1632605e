"""TextSGC one-hop precompute on the HIP engine vs
the reference's own function's outputs (tests/golden/gen_textsgc.py), bit for
bit: the SpMM (S . S[:, split]) is the product kernel; transpose, min/max,
useful-column filter and scaling are device torch ops."""
import os

import numpy as np
import pytest
import scipy.sparse as sp
import torch

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "textsgc_case.npz")


def _case():
    z = np.load(GOLDEN)
    n = int(z["n"])
    S = sp.csr_matrix((z["data"], z["indices"], z["indptr"]), shape=(n, n))
    idx = {k: list(z[f"idx_{k}"]) for k in ("train", "val", "test")}
    return z, S, idx


def test_textsgc_precompute_bit_exact():
    from sgc_amd.textsgc import sgc_precompute, sparse_to_torch_dense, sparse_to_torch_sparse
    z, S, idx = _case()
    adj = sparse_to_torch_sparse(S, device="cuda")
    dense = sparse_to_torch_dense(S, device="cpu")  # train.py:104 builds it on the host
    feats, secs = sgc_precompute(adj, dense, 1, idx)
    assert secs > 0
    assert feats["train"].is_cuda and not feats["val"].is_cuda and not feats["test"].is_cuda
    for k in ("train", "val", "test"):
        got = feats[k].cpu().numpy()
        want = z[f"feat_{k}"]
        assert got.shape == want.shape, k
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), k


def test_textsgc_rejects_degree_and_cpu_adj():
    from sgc_amd.textsgc import sgc_precompute, sparse_to_torch_dense, sparse_to_torch_sparse
    _, S, idx = _case()
    dense = sparse_to_torch_dense(S, device="cpu")
    with pytest.raises(AssertionError):
        sgc_precompute(sparse_to_torch_sparse(S, device="cuda"), dense, 2, idx)
    with pytest.raises(RuntimeError):
        sgc_precompute(sparse_to_torch_sparse(S, device="cpu"), dense, 1, idx)
