"""The drop-in on CPU tensors (the reference's --no-cuda mode, args.py:39):
sgc_precompute / spmm run on libsgc_amd.so's host twin (sgc_*_cpu), SGC's
forward is the reference's own nn.Linear arithmetic.  Everything here is
bit-exact against fixtures the reference itself produced (tests/golden), and
runs without a GPU.  The oracle is never imported by the product path; here
it is not used at all -- the goldens are the reference's outputs.
"""
import hashlib
import json
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def bits_equal(a, b):
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.fixture(scope="module", autouse=True)
def _lib_built():
    from sgc_amd import build
    build.build(verbose=False)


def coo_cpu(c):
    n = int(c["n"])
    idx = torch.from_numpy(np.stack([c["rows"], c["cols"]]).astype(np.int64))
    return torch.sparse_coo_tensor(idx, torch.from_numpy(c["vals"]), (n, n))


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_tiny_cases_cpu_bit_exact(tiny_cases, threads):
    """All 17 reference cases (unsorted COO with duplicates, empty rows, hub
    rows, special values, K = 0..3) through the drop-in on CPU tensors."""
    from sgc_amd.utils import sgc_precompute
    saved = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        for name, c in tiny_cases.items():
            adj = coo_cpu(c)
            X = torch.from_numpy(c["X"])
            for key in sorted(k for k in c if k.startswith("Y")):
                K = int(key[1:])
                out, secs = sgc_precompute(X, adj, K)
                if K == 0:
                    assert out is X
                    continue
                assert out.device.type == "cpu" and secs >= 0
                assert bits_equal(out.numpy(), c[key]), (name, K, threads)
    finally:
        torch.set_num_threads(saved)


@pytest.mark.parametrize("shape", ["cora", "pubmed"])
def test_shape_hashes_cpu(shape, shapes_golden, shape_rows):
    from sgc_amd import graphs
    from sgc_amd.utils import sgc_precompute
    g = shapes_golden[shape]
    S = graphs.synthetic_graph(shape, seed=g["seed"])
    rows, cols, vals = S.coo()
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.stack([rows, cols])),
                                  torch.from_numpy(vals), (S.n, S.n))
    X = torch.from_numpy(graphs.synthetic_features(shape, g["n"], g["features"],
                                                   seed=g["feature_seed"]))
    for K, rec in g["outputs"].items():
        Y, _ = sgc_precompute(X, adj, int(K))
        Y = Y.numpy()
        assert bits_equal(Y[shape_rows[f"{shape}_rows"]], shape_rows[f"{shape}_K{K}"]), (shape, K)
        assert sha(Y) == rec["sha"], (shape, K)


def test_cpu_csr_and_row_slices(tiny_cases):
    """CSR-layout adjacency, row-range SpMM with padded strides, no writes past F."""
    from sgc_amd.propagate import DeviceCSR, spmm
    from sgc_amd.utils import sgc_precompute
    c = tiny_cases["norm_n48_F602"]
    adj = coo_cpu(c)
    out, _ = sgc_precompute(torch.from_numpy(c["X"]), adj.to_sparse_csr(), 2)
    assert bits_equal(out.numpy(), c["Y2"])
    csr = DeviceCSR.from_torch(adj)
    assert csr.device.type == "cpu"
    X = torch.from_numpy(c["X"])
    Xpad = torch.zeros((X.shape[0], 640))
    Xpad[:, :602] = X
    for lo, hi in ((0, 5), (5, 31), (31, 48), (10, 10)):
        for Xin in (X, Xpad[:, :602]):
            o = torch.full((hi - lo, 700), float("nan"))
            spmm(csr, Xin, lo, hi, out=o[:, :602])
            assert bits_equal(o[:, :602].numpy(), c["Y1"][lo:hi])
            assert torch.isnan(o[:, 602:]).all()


def test_cpu_ingest_matches_stable_row_sort(tiny_cases):
    from sgc_amd.propagate import STATUS_COLS_ASCENDING, STATUS_ROWS_SORTED, DeviceCSR
    c = tiny_cases["raw_unsorted_dups_F7"]
    csr = DeviceCSR.from_torch(coo_cpu(c))
    assert not csr.status & STATUS_ROWS_SORTED
    order = np.argsort(c["rows"], kind="stable")
    assert np.array_equal(csr.col_idx.numpy(), c["cols"][order])
    assert bits_equal(csr.val.numpy(), c["vals"][order])
    assert np.array_equal(csr.row_ptr.numpy(),
                          np.concatenate([[0], np.cumsum(np.bincount(c["rows"], minlength=int(c["n"])))]))
    c = tiny_cases["norm_n48_F64"]
    csr = DeviceCSR.from_torch(coo_cpu(c))
    assert csr.status & STATUS_ROWS_SORTED and csr.status & STATUS_COLS_ASCENDING


def test_cpu_errors_are_loud():
    from sgc_amd._lib import SGCError
    from sgc_amd.utils import sgc_precompute
    adj = torch.sparse_coo_tensor(torch.tensor([[0, 1], [1, 0]]), torch.tensor([1.0, 1.0]), (2, 2))
    with pytest.raises(RuntimeError):
        sgc_precompute(torch.ones(5, 3), adj, 1)  # size mismatch
    bad = torch.sparse_coo_tensor(torch.tensor([[0, 1], [1, 7]]), torch.tensor([1.0, 2.0]), (3, 3),
                                  check_invariants=False)
    with pytest.raises(SGCError):
        sgc_precompute(torch.zeros((3, 4)), bad, 1)
    with pytest.raises(TypeError):
        sgc_precompute(torch.zeros((2, 4)), adj.double(), 1)


def test_sgc_forward_cpu_is_reference_linear():
    from sgc_amd.models import SGC, sgc_cross_entropy
    torch.manual_seed(0)
    m = SGC(30, 5)
    x = torch.randn(40, 30)
    assert torch.equal(m(x), torch.nn.functional.linear(x, m.W.weight, m.W.bias))
    y = torch.randint(0, 5, (40,))
    loss = sgc_cross_entropy(m, x, y)
    loss.backward()
    assert m.W.weight.grad is not None


def test_citation_driver_no_cuda_reproduces_reference(tmp_path, monkeypatch):
    """drivers/citation.py --no-cuda on the synthetic Planetoid dataset: the
    propagated features hash and the printed accuracies equal what the
    reference's own citation.py printed on the same files (gen_e2e.py)."""
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "drivers"))
    try:
        from planetoid_synth import write_planetoid
        import citation
        from sgc_amd.utils import load_citation, sgc_precompute
        with open(os.path.join(HERE, "golden", "e2e_citation.json")) as f:
            golden = json.load(f)
        write_planetoid(str(tmp_path), **golden["dataset"])
        monkeypatch.chdir(tmp_path)
        g = golden["reference_load_and_precompute"]
        adj, feats, *_ = load_citation("synth", "AugNormAdj", False)
        assert sha(adj._indices().numpy()) == g["sha_adj_indices"]
        assert sha(adj._values().numpy()) == g["sha_adj_values"]
        y, _ = sgc_precompute(feats, adj, 2)
        assert sha(y.numpy()) == g["sha_precompute_K2"]
        ref = golden["reference_citation_py"]
        assert "--no-cuda" in ref["args"]
        acc_val, acc_test = citation.main(ref["args"])
        assert round(acc_val, 4) == ref["val_acc"] and round(acc_test, 4) == ref["test_acc"]
    finally:
        sys.path.remove(HERE)
        sys.path.pop(0)
