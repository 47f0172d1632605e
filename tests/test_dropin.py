"""Host-side drop-in surface (no GPU): normalisation, format conversion,
loaders, args, metrics, model construction, and loud failure off-GPU.

Where /root/reference exists (the build container) the reference's own
modules are imported and compared against directly; on the GPU box those
comparisons skip and the committed golden hashes (test_oracle.py) carry the
parity.  Loader tests read only Planetoid-format files this test writes.
"""
import os
import pickle
import sys

import numpy as np
import pytest
import scipy.sparse as sp
import torch

REF = os.environ.get("SGC_REFERENCE", "/root/reference")
HAVE_REF = os.path.isdir(REF) and os.path.exists(os.path.join(REF, "utils.py"))
needs_ref = pytest.mark.skipif(not HAVE_REF, reason="reference tree not present")


@pytest.fixture(scope="module")
def ref():
    """The reference's normalization/utils/metrics/args modules, imported
    under private names so they cannot shadow anything."""
    import importlib.util
    mods = {}
    sys.path.insert(0, REF)  # reference utils does `from normalization import ...`
    saved = {k: sys.modules.get(k) for k in ("normalization", "utils", "metrics", "args")}
    try:
        for name in ("normalization", "utils", "metrics", "args"):
            spec = importlib.util.spec_from_file_location(name, os.path.join(REF, f"{name}.py"))
            m = importlib.util.module_from_spec(spec)
            sys.modules[name] = m
            sys.dont_write_bytecode = True
            spec.loader.exec_module(m)
            mods[name] = m
    finally:
        sys.path.remove(REF)
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    return mods


def _rand_adj(rng, n, m, weighted=False, selfloops=False):
    r, c = rng.integers(0, n, m), rng.integers(0, n, m)
    if not selfloops:
        keep = r != c
        r, c = r[keep], c[keep]
    v = rng.integers(1, 3, r.shape[0]).astype(np.float64) if weighted else np.ones(r.shape[0])
    return sp.coo_matrix((v, (r, c)), shape=(n, n))


@needs_ref
@pytest.mark.parametrize("kind", ["binary_sym", "weighted", "selfloops", "coo_unsorted", "empty"])
def test_aug_normalized_adjacency_matches_reference(ref, kind):
    from sgc_amd.normalization import aug_normalized_adjacency
    rng = np.random.default_rng(5)
    n = 300
    if kind == "binary_sym":
        A = _rand_adj(rng, n, 2000).tocsr()
        A = A + A.T
        A.data[:] = 1
    elif kind == "weighted":
        A = _rand_adj(rng, n, 2000, weighted=True).tocsr()
        A = A + A.T
    elif kind == "selfloops":
        A = _rand_adj(rng, n, 2000, selfloops=True).tocsr()
    elif kind == "coo_unsorted":
        A = _rand_adj(rng, n, 2000)  # raw COO with duplicates, unsorted
    else:
        A = sp.csr_matrix((n, n))
    got = aug_normalized_adjacency(A)
    want = ref["normalization"].aug_normalized_adjacency(A)
    assert np.array_equal(got.row, want.row) and np.array_equal(got.col, want.col)
    assert np.array_equal(got.data.view(np.uint64), want.data.view(np.uint64))


@needs_ref
def test_row_normalize_and_fetch(ref):
    from sgc_amd.normalization import fetch_normalization, row_normalize
    rng = np.random.default_rng(2)
    X = sp.random(50, 30, density=0.2, random_state=3, format="lil")
    X[3, :] = 0
    a = row_normalize(X).toarray()
    b = ref["normalization"].row_normalize(X).toarray()
    assert np.array_equal(a, b)
    bad_mine, bad_ref = fetch_normalization("NormLap"), ref["normalization"].fetch_normalization("NormLap")
    with pytest.raises(TypeError):
        bad_mine(sp.eye(3))
    with pytest.raises(TypeError):
        bad_ref(sp.eye(3))
    del rng


@needs_ref
def test_sparse_mx_to_torch_matches_reference(ref):
    from sgc_amd.normalization import aug_normalized_adjacency
    from sgc_amd.utils import sparse_mx_to_torch_sparse_tensor
    rng = np.random.default_rng(9)
    S = aug_normalized_adjacency(_rand_adj(rng, 100, 500))
    a = sparse_mx_to_torch_sparse_tensor(S)
    b = ref["utils"].sparse_mx_to_torch_sparse_tensor(S)
    assert torch.equal(a._indices(), b._indices())
    assert torch.equal(a._values(), b._values())
    assert a.shape == b.shape and a.dtype == b.dtype and not a.is_coalesced()


def _write_planetoid(root, name, rng, n_train=20, n_val_extra=520, n_test=100, F=40, C=4,
                     isolated=False):
    """A tiny Planetoid-format dataset (the files this test itself writes)."""
    data = os.path.join(root, "data")
    os.makedirs(data, exist_ok=True)
    n_all = n_train + n_val_extra
    n_total = n_all + n_test

    def feats(m):
        return sp.csr_matrix((rng.random((m, F)) < 0.2).astype(np.float32))

    def labels(m):
        y = np.zeros((m, C))
        y[np.arange(m), rng.integers(0, C, m)] = 1
        return y

    test_idx = rng.permutation(np.arange(n_all, n_total))
    if isolated:  # citeseer quirk: a hole in the test index range
        test_idx = test_idx[test_idx != n_all + 5]
    graph = {i: [int(j) for j in rng.integers(0, n_total, 3) if j != i] for i in range(n_total)}
    objs = {"x": feats(n_train), "y": labels(n_train), "allx": feats(n_all), "ally": labels(n_all),
            "tx": feats(len(test_idx)), "ty": labels(len(test_idx)), "graph": graph}
    for k, v in objs.items():
        with open(os.path.join(data, f"ind.{name}.{k}"), "wb") as f:
            pickle.dump(v, f)
    with open(os.path.join(data, f"ind.{name}.test.index"), "w") as f:
        f.write("\n".join(str(int(i)) for i in test_idx))


@needs_ref
@pytest.mark.parametrize("name", ["cora", "citeseer"])
def test_load_citation_matches_reference(ref, tmp_path, monkeypatch, name):
    from sgc_amd.utils import load_citation
    _write_planetoid(str(tmp_path), name, np.random.default_rng(1), isolated=(name == "citeseer"))
    monkeypatch.chdir(tmp_path)
    a = load_citation(name, "AugNormAdj", cuda=False)
    b = ref["utils"].load_citation(name, "AugNormAdj", cuda=False)
    assert torch.equal(a[0]._indices(), b[0]._indices())
    assert torch.equal(a[0]._values(), b[0]._values())
    for x, y in zip(a[1:], b[1:]):
        assert torch.equal(x, y)


def test_load_reddit_npz_roundtrip(tmp_path, monkeypatch):
    """Reddit loader on an npz dataset (no pickles); quirk: a non-directory
    data_path (reddit.py:38 passes the normalisation name) reads data/."""
    from sgc_amd.utils import load_reddit_data
    rng = np.random.default_rng(0)
    n, F = 60, 12
    data = tmp_path / "data"
    data.mkdir()
    A = _rand_adj(rng, n, 200).tocsr()
    A.data[:] = 1
    sp.save_npz(str(data / "reddit_adj.npz"), A)
    idx = rng.permutation(n)
    tr, va, te = idx[:30], idx[30:45], idx[45:]
    np.savez(str(data / "reddit.npz"), feats=rng.standard_normal((n, F)), y_train=rng.integers(0, 5, 30),
             y_val=rng.integers(0, 5, 15), y_test=rng.integers(0, 5, 15), train_index=tr,
             val_index=va, test_index=te)
    monkeypatch.chdir(tmp_path)
    adj, train_adj, feats, labels, i_tr, i_va, i_te = load_reddit_data("AugNormAdj", cuda=False)
    assert adj.shape == (n, n) and train_adj.shape == (30, 30)
    assert feats.shape == (n, F) and torch.allclose(feats.mean(0), torch.zeros(F), atol=1e-5)
    assert np.array_equal(i_tr, tr)
    assert labels.dtype == torch.int64


@needs_ref
def test_args_defaults_match_reference(ref, monkeypatch):
    from sgc_amd.args import get_citation_args
    monkeypatch.setattr(sys, "argv", ["citation.py"])
    assert vars(get_citation_args()) == vars(ref["args"].get_citation_args())
    monkeypatch.setattr(sys, "argv", ["citation.py", "--dataset", "citeseer", "--tuned", "--degree", "3"])
    assert vars(get_citation_args()) == vars(ref["args"].get_citation_args())


@needs_ref
def test_metrics_match_reference(ref):
    from sgc_amd.metrics import accuracy, f1
    g = torch.Generator().manual_seed(0)
    out = torch.randn(200, 7, generator=g)
    lab = torch.randint(0, 7, (200,), generator=g)
    assert torch.equal(accuracy(out, lab), ref["metrics"].accuracy(out, lab))
    assert f1(out, lab) == ref["metrics"].f1(out, lab)


def test_model_surface():
    from sgc_amd.models import SGC, get_model
    m = get_model("SGC", 20, 3, cuda=False)
    assert isinstance(m, SGC) and isinstance(m.W, torch.nn.Linear)
    assert m.W.weight.shape == (3, 20) and m.W.bias.shape == (3,)
    with pytest.raises(NotImplementedError):
        get_model("MLP", 20, 3, cuda=False)
    with pytest.raises(NotImplementedError):
        get_model("GCN", 20, 3, cuda=False)


def test_cpu_tensors_run_like_the_reference():
    """CPU tensors take the library's host twin (reference --no-cuda mode,
    args.py:39), not an error; K=0 returns the input object."""
    from sgc_amd.models import SGC
    from sgc_amd.utils import sgc_precompute
    adj = torch.sparse_coo_tensor(torch.tensor([[0, 1], [1, 0]]), torch.tensor([1.0, 1.0]), (2, 2))
    X = torch.arange(6, dtype=torch.float32).reshape(2, 3)
    out, _ = sgc_precompute(X, adj, 1)
    assert torch.equal(out, torch.spmm(adj, X))
    out, _ = sgc_precompute(X, adj, 0)  # K=0: the input object, as the reference
    assert out is X
    m = SGC(3, 2)
    assert torch.equal(m(X), m.W(X))


def test_dropin_modules_reexport():
    import importlib
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "dropin"))
    try:
        for name, attrs in {"utils": ["load_citation", "load_reddit_data", "sgc_precompute", "set_seed",
                                      "sparse_mx_to_torch_sparse_tensor"],
                            "models": ["SGC", "get_model"], "metrics": ["accuracy", "f1"],
                            "args": ["get_citation_args"],
                            "normalization": ["fetch_normalization", "row_normalize",
                                              "aug_normalized_adjacency"]}.items():
            spec = importlib.util.spec_from_file_location(
                f"dropin_{name}", os.path.join(sys.path[0], f"{name}.py"))
            m = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(m)
            for a in attrs:
                assert getattr(m, a).__module__.startswith("sgc_amd"), (name, a)
    finally:
        sys.path.pop(0)


def test_cross_entropy_routing_rules():
    """SGCLogits routes only the plain F.cross_entropy form to the HIP loss
    (sgc_amd.models._cross_entropy_args): ROCm float32 [M, C <= 64] logits,
    int64 [M] labels on the same device, mean reduction, no weights, no
    smoothing; everything else -- CPU tensors here -- is torch's own call."""
    import torch
    from sgc_amd.models import SGCLogits, _cross_entropy_args
    x = torch.randn(6, 5)
    y = torch.randint(0, 5, (6,))
    assert _cross_entropy_args((x, y), {}) is None  # CPU tensors: torch's path
    ref = torch.nn.functional.cross_entropy(x, y)
    got = torch.nn.functional.cross_entropy(x.as_subclass(SGCLogits), y)
    assert type(got) is torch.Tensor and torch.equal(got, ref)
    got = torch.nn.functional.cross_entropy(x.as_subclass(SGCLogits), y, reduction="sum")
    assert torch.equal(got, torch.nn.functional.cross_entropy(x, y, reduction="sum"))
    # non-plain forms are refused before any device check
    for kw in ({"weight": torch.ones(5)}, {"reduction": "none"}, {"label_smoothing": 0.1},
               {"size_average": False}, {"bogus": 1}):
        assert _cross_entropy_args((x, y), kw) is None
    assert _cross_entropy_args((x, y.to(torch.int32)), {}) is None
    out = x.as_subclass(SGCLogits)
    assert type(out.max(1)[1]) is torch.Tensor and type(out + 1) is torch.Tensor
