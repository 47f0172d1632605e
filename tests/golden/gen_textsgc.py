"""Golden vectors for the TextSGC one-hop precompute,
made by RUNNING THE REFERENCE'S OWN FUNCTIONS on CPU.

    python tests/golden/gen_textsgc.py          # in the build container

The reference module /root/reference/downstream/TextSGC/utils.py does not
import here: its first lines import scipy.sparse.linalg.eigen.arpack, which
scipy 1.15 no longer has (an ordinary ImportError of an unrelated symbol).
So this script reads that file as text, takes the three functions on the
precompute path out of it with `ast` -- sparse_to_torch_sparse (:103-118),
sparse_to_torch_dense (:120-123), sgc_precompute (:131-152) -- and executes
exactly those definitions with numpy/torch/perf_counter in scope.  The
reference moves tensors with .cuda(); there is no GPU in this container, so
while the function runs Tensor.cuda returns the tensor itself (CPU), i.e. the
reference's arithmetic is torch.spmm's CPU kernel -- the oracle semantics of
this build.  Nothing of the reference is written to the
repo: only the inputs and outputs below.

Input: a seeded TextGCN-shaped graph (doc-word TF-IDF edges, word-word PMI
edges, self loops, symmetric normalisation, plus isolated word nodes whose
features have zero range over the training docs and must be filtered).
Output: tests/golden/textsgc_case.npz.
"""
import ast
import os
import sys
from time import perf_counter

import numpy as np
import scipy.sparse as sp
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("SGC_REFERENCE", "/root/reference")
SRC = os.path.join(REF, "downstream", "TextSGC", "utils.py")
WANT = ("sparse_to_torch_sparse", "sparse_to_torch_dense", "sgc_precompute")


def reference_functions():
    tree = ast.parse(open(SRC).read(), SRC)
    defs = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in WANT]
    assert sorted(d.name for d in defs) == sorted(WANT), [d.name for d in defs]
    ns = {"np": np, "torch": torch, "perf_counter": perf_counter}
    exec(compile(ast.Module(body=defs, type_ignores=[]), SRC, "exec"), ns)
    return ns


def text_graph(n_docs=240, n_words=420, n_isolated=12, seed=7):
    """Normalised TextGCN-style adjacency, fp64 CSR (the shape load_corpus returns)."""
    rng = np.random.default_rng(seed)
    n = n_docs + n_words + n_isolated
    rows, cols, vals = [], [], []
    for d in range(n_docs):  # doc-word TF-IDF
        ws = rng.choice(n_words, size=rng.integers(4, 25), replace=False)
        rows += [d] * len(ws)
        cols += list(n_docs + ws)
        vals += list(rng.uniform(0.05, 1.0, len(ws)))
    m = 2500  # word-word PMI (positive)
    a, b = rng.integers(0, n_words, m), rng.integers(0, n_words, m)
    keep = a != b
    rows += list(n_docs + a[keep])
    cols += list(n_docs + b[keep])
    vals += list(rng.uniform(0.01, 3.0, keep.sum()))
    A = sp.coo_matrix((vals, (rows, cols)), shape=(n, n)).tocsr()
    A = A.maximum(A.T) + sp.eye(n)
    d = np.asarray(A.sum(1)).ravel() ** -0.5
    S = sp.diags(d) @ A @ sp.diags(d)
    S = sp.csr_matrix(S)
    S.sum_duplicates()
    S.sort_indices()
    perm = rng.permutation(n_docs)
    index_dict = {"train": np.sort(perm[:150]), "val": np.sort(perm[150:190]),
                  "test": perm[190:]}  # test ids deliberately unsorted
    return S, index_dict


def main():
    ref = reference_functions()
    S, index_dict = text_graph()
    adj = ref["sparse_to_torch_sparse"](S, device="cpu")
    dense = ref["sparse_to_torch_dense"](S, device="cpu")
    saved = torch.Tensor.cuda
    torch.Tensor.cuda = lambda self, *a, **k: self  # no GPU here: run on CPU
    try:
        feats, _ = ref["sgc_precompute"](adj, dense, 1, {k: list(v) for k, v in index_dict.items()})
    finally:
        torch.Tensor.cuda = saved
    out = {"indptr": S.indptr.astype(np.int64), "indices": S.indices.astype(np.int64),
           "data": S.data.astype(np.float64), "n": np.int64(S.shape[0])}
    for k, v in index_dict.items():
        out[f"idx_{k}"] = np.asarray(v, dtype=np.int64)
        out[f"feat_{k}"] = feats[k].numpy()
    np.savez_compressed(os.path.join(HERE, "textsgc_case.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    sys.dont_write_bytecode = True
    main()
