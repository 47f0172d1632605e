"""A learnable synthetic Planetoid-format dataset (test data this repo writes).

Planted partition: C communities, edges mostly inside a community, bag-of-
words features drawn from community-specific word distributions, labels =
community.  Files follow the Planetoid layout the reference's load_citation
reads (utils.py:32-90): data/ind.<name>.{x,y,tx,ty,allx,ally,graph} (pickles
of scipy/numpy/dict objects written HERE) and data/ind.<name>.test.index.
Deterministic in `seed`, so the GPU box regenerates identical files.
"""
import os
import pickle

import numpy as np
import scipy.sparse as sp


def write_planetoid(root, name="synth", n=1200, n_feat=300, n_class=5, n_train=100, n_test=300,
                    avg_deg=4, p_in=0.6, words_per_doc=12, p_own=0.3, seed=7):
    rng = np.random.default_rng(seed)
    comm = rng.integers(0, n_class, n)
    # edges: endpoints in the same community with prob p_in
    m = n * avg_deg // 2
    u = rng.integers(0, n, m)
    same = rng.random(m) < p_in
    v = np.empty(m, np.int64)
    for i in range(m):
        if same[i]:
            members = np.flatnonzero(comm == comm[u[i]])
            v[i] = members[rng.integers(0, members.size)]
        else:
            v[i] = rng.integers(0, n)
    graph = {i: [] for i in range(n)}
    for a, b in zip(u.tolist(), v.tolist()):
        if a != b:
            graph[a].append(b)
    # features: each community prefers its own block of words
    block = n_feat // n_class
    X = np.zeros((n, n_feat), np.float32)
    for i in range(n):
        c = comm[i]
        own = rng.random(words_per_doc) < p_own
        w = np.where(own, c * block + rng.integers(0, block, words_per_doc),
                     rng.integers(0, n_feat, words_per_doc))
        X[i, w] = 1.0
    Y = np.eye(n_class)[comm]
    # Planetoid split: allx/ally = first n - n_test nodes, tx/ty = the rest
    # (stored in a shuffled test.index order), x/y = the first n_train
    n_all = n - n_test
    test_idx = np.arange(n_all, n)
    test_order = rng.permutation(test_idx)
    objs = {
        "x": sp.csr_matrix(X[:n_train]), "y": Y[:n_train],
        "allx": sp.csr_matrix(X[:n_all]), "ally": Y[:n_all],
        "tx": sp.csr_matrix(X[test_idx]), "ty": Y[test_idx], "graph": graph,
    }
    data = os.path.join(root, "data")
    os.makedirs(data, exist_ok=True)
    for k, obj in objs.items():
        with open(os.path.join(data, f"ind.{name}.{k}"), "wb") as f:
            pickle.dump(obj, f)
    # load_citation reorders features[test_idx_reorder] = features[sorted]: the
    # file lists the test nodes in `test_order`; store tx/ty in that order.
    with open(os.path.join(data, f"ind.{name}.tx"), "wb") as f:
        pickle.dump(sp.csr_matrix(X[test_order]), f)
    with open(os.path.join(data, f"ind.{name}.ty"), "wb") as f:
        pickle.dump(Y[test_order], f)
    with open(os.path.join(data, f"ind.{name}.test.index"), "w") as f:
        f.write("\n".join(str(int(i)) for i in test_order))
    return dict(n=n, n_feat=n_feat, n_class=n_class, n_train=n_train, n_test=n_test,
                avg_deg=avg_deg, p_in=p_in, words_per_doc=words_per_doc, p_own=p_own, seed=seed)
