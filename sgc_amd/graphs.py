"""Seeded synthetic graphs of the shapes BASELINE.json names (host side, numpy).

The reference's real inputs (Planetoid pickles, reddit_adj.npz) are either
absent from the reference tree or are pickles, which this build never loads
from the reference.  BASELINE.json's metric is quoted on *synthetic CSR graphs
of Cora/Pubmed/Reddit shape*; SURVEY.md section 8(d) fixes the recipe:

* undirected, unique, non-self pairs drawn by R-MAT(a=.57, b=.19, c=.19,
  d=.05) over 2**ceil(log2 N) ids, ids >= N rejected, vertices relabelled by a
  random permutation;
* A = U + U^T (binary), S = AugNorm(A) = (D+I)^-1/2 (A+I) (D+I)^-1/2 in fp64,
  rounded once to fp32 (reference normalization.py:5-12, utils.py:23-30).

Everything is a pure function of (shape, seed) through numpy's PCG64, so the
GPU box regenerates bit-identical inputs; tests/golden pins the hashes.
"""
from dataclasses import dataclass

import numpy as np

# (nodes, unique undirected non-self edges, features, hops) -- SURVEY.md 8(d).
# nnz(S) = 2 * edges + nodes: Cora 13,264; Pubmed 108,365 (edges chosen so the
# synthetic nnz equals the real one); Reddit 23,446,803; RMAT 260,194,304.
SHAPES = {
    "cora": dict(n=2708, edges=5278, features=1433, hops=2),
    "pubmed": dict(n=19717, edges=44324, features=500, hops=2),
    "reddit": dict(n=232965, edges=11606919, features=602, hops=2),
    "rmat": dict(n=4194304, edges=128000000, features=256, hops=3),
}


@dataclass
class CSRGraph:
    """Normalised adjacency S in CSR (int32 indices, fp32 values, rows sorted
    by column, no duplicates -- the layout the reference produces)."""
    n: int
    row_ptr: np.ndarray  # int32 [n+1]
    col_idx: np.ndarray  # int32 [nnz]
    val: np.ndarray      # float32 [nnz]

    @property
    def nnz(self):
        return int(self.row_ptr[-1])

    def coo(self):
        rows = np.repeat(np.arange(self.n, dtype=np.int64), np.diff(self.row_ptr))
        return rows, self.col_idx.astype(np.int64), self.val


def rmat_pairs(n, n_edges, seed=0, a=0.57, b=0.19, c=0.19, batch=None):
    """Unique undirected non-self pairs (lo < hi) from R-MAT, relabelled.

    Returns int64 arrays (u, v), sorted by the relabelled key u*n+v order of
    the *pre-relabel* selection (deterministic given the seed)."""
    rng = np.random.default_rng(seed)
    scale = max(1, int(np.ceil(np.log2(max(n, 2)))))
    keys = np.empty(0, np.int64)
    batch = batch or max(1 << 16, int(n_edges * 1.4))
    ab, abc = a + b, a + b + c
    while keys.shape[0] < n_edges:
        u = np.zeros(batch, np.int64)
        v = np.zeros(batch, np.int64)
        for lvl in range(scale):
            r = rng.random(batch)
            u |= (r >= ab).astype(np.int64) << lvl
            v |= (((r >= a) & (r < ab)) | (r >= abc)).astype(np.int64) << lvl
        ok = (u < n) & (v < n) & (u != v)
        u, v = u[ok], v[ok]
        lo, hi = np.minimum(u, v), np.maximum(u, v)
        keys = np.unique(np.concatenate([keys, lo * n + hi]))
    if keys.shape[0] > n_edges:
        keys = np.sort(rng.choice(keys, size=n_edges, replace=False))
    perm = rng.permutation(n).astype(np.int64)
    u, v = perm[keys // n], perm[keys % n]
    return np.minimum(u, v), np.maximum(u, v)


def aug_norm_csr_from_pairs(n, u, v):
    """S = AugNorm(U + U^T) for unique non-self undirected pairs, in CSR.

    Fast numpy restatement of normalization.py:5-12 for a binary symmetric A
    without self loops: every entry of A+I is 1.0, rowsum = deg+1 (exact in
    fp64), d = rowsum**-0.5 (np.power, as normalization.py:8), value =
    (d_i * 1.0) * d_j in fp64 (the dia.csr.dia product of :12), then one
    rounding to fp32 (utils.py:25).  Entries sorted by (row, col): the
    scipy .tocoo() order the reference hands to torch."""
    rows = np.concatenate([u, v, np.arange(n, dtype=np.int64)])
    cols = np.concatenate([v, u, np.arange(n, dtype=np.int64)])
    key = rows * n + cols
    key.sort(kind="stable")
    rows = key // n
    cols = key - rows * n
    counts = np.bincount(rows, minlength=n)
    rowsum = counts.astype(np.float64)
    with np.errstate(divide="ignore"):
        d = np.power(rowsum, -0.5)
    d[np.isinf(d)] = 0.0
    val = ((d[rows] * 1.0) * d[cols]).astype(np.float32)
    row_ptr = np.zeros(n + 1, np.int64)
    np.cumsum(counts, out=row_ptr[1:])
    if row_ptr[-1] >= 2**31 or n >= 2**31:
        raise ValueError("graph too large for int32 CSR")
    return CSRGraph(n, row_ptr.astype(np.int32), cols.astype(np.int32), val)


def synthetic_graph(shape, seed=0, n=None, edges=None):
    spec = dict(SHAPES[shape])
    n = n or spec["n"]
    edges = edges or spec["edges"]
    u, v = rmat_pairs(n, edges, seed=seed)
    return aug_norm_csr_from_pairs(n, u, v)


def synthetic_features(shape, n, F, seed=1):
    """Features of the named shape.

    cora   : binary bag-of-words (~1.27 % dense), row-normalised (normalization.py:21-28)
    pubmed : 10 %-dense U(0.002, 1.26) TF-IDF-like, row-normalised
    reddit/rmat : N(0,1), column-standardised as utils.py:119 (unbiased std)
    """
    rng = np.random.default_rng(seed)
    if shape in ("cora", "pubmed"):
        density = 0.0127 if shape == "cora" else 0.10
        mask = rng.random((n, F)) < density
        if shape == "cora":
            X = mask.astype(np.float64)
        else:
            X = np.where(mask, rng.uniform(0.002, 1.26, (n, F)), 0.0)
        rs = X.sum(1)
        with np.errstate(divide="ignore"):
            r_inv = np.power(rs, -1.0)
        r_inv[np.isinf(r_inv)] = 0.0
        return (X * r_inv[:, None]).astype(np.float32)
    X = rng.standard_normal((n, F), dtype=np.float32)
    mu = X.mean(axis=0, dtype=np.float64)
    sd = X.std(axis=0, ddof=1, dtype=np.float64)
    return ((X - mu.astype(np.float32)) / sd.astype(np.float32)).astype(np.float32)
