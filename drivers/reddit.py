"""Reddit driver on the MI355X engine -- counterpart of the reference's
reddit.py (same flags and output line), reading data/reddit_adj.npz and
data/reddit.npz like the reference.

    python drivers/reddit.py [--inductive] [--test] [--degree 2] [--epochs 2]

Flow (reference reddit.py:12-74): seed -> load_reddit_data (A + A^T, train
subgraph, AugNorm, standardised features) -> SGC(602, 41) -> sgc_precompute
on the full graph (timed) and, with --inductive, on the train subgraph ->
LBFGS(lr=1) -> micro-F1.  --synthetic N builds a seeded Reddit-shape graph
instead of reading data/ (the real Reddit data is not distributed with the
reference).
"""
import argparse
import os
import sys
from time import perf_counter

import numpy as np
import torch
import torch.nn.functional as F
import torch.optim as optim

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sgc_amd.metrics import f1  # noqa: E402
from sgc_amd.models import SGC  # noqa: E402
from sgc_amd.utils import load_reddit_data, set_seed, sgc_precompute  # noqa: E402

NORMALIZATIONS = ["NormLap", "Lap", "RWalkLap", "FirstOrderGCN", "AugNormAdj", "NormAdj", "RWalk",
                  "AugRWalk", "NoNorm"]


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--no-cuda", action="store_true", default=False, help="Disables CUDA training.")
    p.add_argument("--inductive", action="store_true", default=False, help="inductive training.")
    p.add_argument("--test", action="store_true", default=False, help="inductive training.")
    p.add_argument("--seed", type=int, default=42, help="Random seed.")
    p.add_argument("--epochs", type=int, default=2, help="Number of epochs to train.")
    p.add_argument("--weight_decay", type=float, default=0, help="Weight decay (L2 loss on parameters).")
    p.add_argument("--normalization", type=str, default="AugNormAdj", choices=NORMALIZATIONS,
                   help="Normalization method for the adjacency matrix.")
    p.add_argument("--model", type=str, default="SGC", help="model to use.")
    p.add_argument("--degree", type=int, default=2, help="degree of the approximation.")
    p.add_argument("--synthetic", type=int, default=0,
                   help="use a seeded Reddit-shape synthetic graph with this many nodes (0: read data/)")
    args = p.parse_args(argv)
    args.cuda = not args.no_cuda and torch.cuda.is_available()
    return args


def synthetic_reddit(n, seed=0):
    """Reddit-shaped stand-in with the reference's preprocessing applied."""
    import scipy.sparse as sp

    from sgc_amd import graphs
    from sgc_amd.normalization import fetch_normalization
    from sgc_amd.utils import sparse_mx_to_torch_sparse_tensor
    spec = graphs.SHAPES["reddit"]
    edges = max(1, int(spec["edges"] * n / spec["n"]))
    u, v = graphs.rmat_pairs(n, edges, seed=seed)
    A = sp.coo_matrix((np.ones(edges), (u, v)), shape=(n, n)).tocsr()
    A = A + A.T
    rng = np.random.default_rng(seed + 7)
    perm = rng.permutation(n)
    tr, va, te = np.sort(perm[: int(0.66 * n)]), np.sort(perm[int(0.66 * n): int(0.76 * n)]), \
        np.sort(perm[int(0.76 * n):])
    feats = torch.from_numpy(rng.standard_normal((n, spec["features"])).astype(np.float32))
    feats = (feats - feats.mean(dim=0)) / feats.std(dim=0)
    labels = torch.from_numpy(rng.integers(0, 41, n))
    norm = fetch_normalization("AugNormAdj")
    adj = sparse_mx_to_torch_sparse_tensor(norm(A)).float()
    train_adj = sparse_mx_to_torch_sparse_tensor(norm(A[tr][:, tr])).float()
    out = (adj.cuda(), train_adj.cuda(), feats.cuda(), labels.cuda(), tr, va, te)
    from sgc_amd.propagate import warmup
    warmup(out[2].device)  # as load_reddit_data does once the data is on the GPU
    return out


def train_regression(model, train_features, train_labels, epochs):
    optimizer = optim.LBFGS(model.parameters(), lr=1)
    model.train()

    def closure():
        optimizer.zero_grad()
        loss = F.cross_entropy(model(train_features), train_labels)
        loss.backward()
        return loss

    t = perf_counter()
    for _ in range(epochs):
        optimizer.step(closure)
    return model, perf_counter() - t


def test_regression(model, test_features, test_labels):
    model.eval()
    return f1(model(test_features), test_labels)


def main(argv=None):
    args = parse(argv)
    set_seed(args.seed, args.cuda)
    if args.synthetic:
        adj, train_adj, features, labels, idx_train, idx_val, idx_test = synthetic_reddit(args.synthetic)
    else:
        adj, train_adj, features, labels, idx_train, idx_val, idx_test = \
            load_reddit_data(args.normalization)
    print("Finished data loading.")
    model = SGC(features.size(1), labels.max().item() + 1)
    if args.cuda:
        model.cuda()
    processed, precompute_time = sgc_precompute(features, adj, args.degree)
    if args.inductive:
        train_features, _ = sgc_precompute(features[idx_train], train_adj, args.degree)
    else:
        train_features = processed[idx_train]
    test_features = processed[idx_test if args.test else idx_val]
    model, train_time = train_regression(model, train_features, labels[idx_train], args.epochs)
    test_f1, _ = test_regression(model, test_features, labels[idx_test if args.test else idx_val])
    print("Total Time: {:.4f}s, {} F1: {:.4f}".format(train_time + precompute_time,
                                                      "Test" if args.test else "Val", test_f1))
    return test_f1, precompute_time, train_time


if __name__ == "__main__":
    main()
