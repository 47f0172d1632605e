"""Generate the golden fixtures under tests/golden/ by running the REFERENCE.

Run in the build container (where /root/reference exists):

    python tests/golden/gen_golden.py

It imports the reference's own modules (/root/reference/normalization.py and
utils.py: aug_normalized_adjacency, sparse_mx_to_torch_sparse_tensor,
sgc_precompute) and runs them on CPU over seeded inputs.  No reference data
file is read (the Planetoid/tuning files are pickles; this build never loads
them) -- graphs and features come from sgc_amd.graphs' seeded generators or
are built inline below.  Outputs:

  tiny_cases.npz      full inputs + outputs of small hand cases (every edge
                      case the engine must keep bit-exact)
  shapes.json         sha256 of S (torch COO indices/values as the reference
                      builds them), of X and of X_K for Cora/Pubmed/Reddit-shape
                      graphs, plus timing of the reference CPU path
  shape_rows.npz      sampled rows of each X_K (readable diffs when a hash fails)

The reference cannot travel to the GPU box; these files do.
"""
import hashlib
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("SGC_REFERENCE", "/root/reference")
sys.path.insert(0, ROOT)
sys.path.insert(0, REF)
sys.dont_write_bytecode = True

import normalization as ref_norm  # noqa: E402  (reference normalization.py)
import utils as ref_utils  # noqa: E402  (reference utils.py)

from sgc_amd import graphs  # noqa: E402

torch.set_num_threads(os.cpu_count() or 1)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def ref_adj(A):
    """S as the reference builds it: normalization.py:5-12 + utils.py:23-30."""
    return ref_utils.sparse_mx_to_torch_sparse_tensor(ref_norm.aug_normalized_adjacency(A)).float()


def ref_prop(X, adj, K):
    out, _ = ref_utils.sgc_precompute(torch.from_numpy(X), adj, K)
    return out.numpy()


def sym_binary(n, pairs):
    u = np.array([p[0] for p in pairs], np.int64)
    v = np.array([p[1] for p in pairs], np.int64)
    A = sp.coo_matrix((np.ones(len(u)), (u, v)), shape=(n, n)).tocsr()
    A = A + A.T
    A.data[:] = 1.0
    return A


def tiny_cases():
    rng = np.random.default_rng(1234)
    cases = {}

    def add(name, rows, cols, vals, n, X, Ks=(0, 1, 2, 3)):
        adj = torch.sparse_coo_tensor(torch.from_numpy(np.stack([rows, cols]).astype(np.int64)),
                                      torch.from_numpy(vals.astype(np.float32)), (n, n))
        d = {"rows": rows.astype(np.int64), "cols": cols.astype(np.int64),
             "vals": vals.astype(np.float32), "n": np.int64(n), "X": X.astype(np.float32)}
        for K in Ks:
            d[f"Y{K}"] = ref_prop(X.astype(np.float32), adj, K)
        cases[name] = d

    def add_norm(name, A, X, Ks=(0, 1, 2, 3)):
        adj = ref_adj(A)
        idx = adj._indices().numpy()
        add(name, idx[0], idx[1], adj._values().numpy(), A.shape[0], X, Ks)

    # random small symmetric graphs through the reference normalisation, F edge widths
    for F in (1, 3, 63, 64, 65, 128, 130, 602):
        n = 48
        pairs = {(int(a), int(b)) for a, b in rng.integers(0, n, (150, 2)) if a != b}
        A = sym_binary(n, sorted(pairs))
        add_norm(f"norm_n48_F{F}", A, rng.standard_normal((n, F)))
    # isolated nodes (rows holding only the +I diagonal) and an all-isolated graph
    A = sym_binary(32, [(0, 1), (1, 2), (5, 9)])
    add_norm("isolated_F17", A, rng.standard_normal((32, 17)))
    add_norm("no_edges_F5", sp.csr_matrix((8, 8)), rng.standard_normal((8, 5)))
    # pre-existing self loops -> diagonal weight 2 after A + I (Citeseer/Pubmed case)
    A = sym_binary(40, [(int(a), int(b)) for a, b in rng.integers(0, 40, (100, 2)) if a != b])
    A = (A + sp.diags(np.where(rng.random(40) < 0.3, 1.0, 0.0))).tocsr()
    add_norm("selfloop_w2_F33", A, rng.standard_normal((40, 33)))
    # weighted A (Reddit's A + A^T doubles edges stored both ways, utils.py:116)
    A = sp.coo_matrix((np.ones(120), (rng.integers(0, 30, 120), rng.integers(0, 30, 120))),
                      shape=(30, 30)).tocsr()
    A = A + A.T
    add_norm("weighted_F9", A, rng.standard_normal((30, 9)))
    # hub row with 1000 nonzeros (heavy-row split path) + light rows
    n = 1100
    hub = np.arange(1, 1001)
    pairs = [(0, int(j)) for j in hub] + [(int(a), int(b)) for a, b in rng.integers(1, n, (600, 2)) if a != b]
    A = sym_binary(n, pairs)
    add_norm("hub1000_F65", A, rng.standard_normal((n, 65)), Ks=(1, 2))
    add_norm("hub1000_F130", A, rng.standard_normal((n, 130)), Ks=(2,))
    # raw COO (not from the normaliser): empty rows, unsorted storage order,
    # duplicate (r,c) entries, zero and negative values
    n = 20
    rows = rng.integers(0, n - 5, 90)  # rows n-5.. stay empty
    cols = rng.integers(0, n, 90)
    rows = np.concatenate([rows, rows[:10]])
    cols = np.concatenate([cols, cols[:10]])  # duplicates
    vals = rng.standard_normal(100)
    vals[::17] = 0.0
    perm = rng.permutation(100)
    add("raw_unsorted_dups_F7", rows[perm], cols[perm], vals[perm], n, rng.standard_normal((n, 7)))
    # lexsorted raw COO with duplicates (sorted rows, non-ascending columns)
    order = np.lexsort((cols, rows))
    add("raw_sorted_dups_F66", rows[order], cols[order], vals[order], n, rng.standard_normal((n, 66)))
    # special values: signed zeros, subnormals, large magnitudes
    n = 16
    pairs = [(i, (i * 7 + 3) % n) for i in range(n)] + [(i, (i + 1) % n) for i in range(n)]
    A = sym_binary(n, pairs)
    X = rng.standard_normal((n, 11)).astype(np.float32)
    X[0, :] = -0.0
    X[1, :] = np.float32(1e-40)  # subnormal
    X[2, :] = np.float32(-3e-39)
    X[3, :] = np.float32(3e38)
    X[4, ::2] = 0.0
    add_norm("special_values_F11", A, X)
    return cases


def shape_case(shape, Ks, seed=0, fseed=1):
    spec = graphs.SHAPES[shape]
    n, E, F = spec["n"], spec["edges"], spec["features"]
    t0 = time.time()
    u, v = graphs.rmat_pairs(n, E, seed=seed)
    A = sp.coo_matrix((np.ones(E), (u, v)), shape=(n, n)).tocsr()
    A = A + A.T  # binary: pairs are unique and lo < hi
    adj = ref_adj(A)
    idx = adj._indices().numpy()
    vals = adj._values().numpy()
    X = graphs.synthetic_features(shape, n, F, seed=fseed)
    gen_s = time.time() - t0
    rec = {"n": n, "edges": E, "features": F, "seed": seed, "feature_seed": fseed,
           "nnz": int(vals.shape[0]), "sha_indices": sha(idx), "sha_values": sha(vals),
           "sha_X": sha(X), "generate_seconds": round(gen_s, 2), "outputs": {}}
    del A, u, v, idx, vals
    rows_pick = np.random.default_rng(99).choice(n, 16, replace=False)
    samples = {f"{shape}_rows": rows_pick}
    adj_t = adj
    for K in Ks:
        # warm-up (allocator first touch); at RMAT scale (260 M nnz, ~31 s per
        # single-threaded COO hop) only on 8 feature columns
        ref_prop(np.ascontiguousarray(X[:, :8]) if n > 10**6 else X, adj_t, 1)
        t0 = time.perf_counter()
        Y = ref_prop(X, adj_t, K)
        dt = time.perf_counter() - t0
        rec["outputs"][str(K)] = {"sha": sha(Y), "ref_cpu_seconds": round(dt, 4),
                                  "ref_cpu_edges_per_s": K * rec["nnz"] / dt}
        samples[f"{shape}_K{K}"] = Y[rows_pick]
    print(shape, json.dumps({k: v for k, v in rec.items() if k != "outputs"}), flush=True)
    return rec, samples


def main():
    """python gen_golden.py [tiny] [cora] [pubmed] [reddit] [rmat]; no argument =
    tiny + cora + pubmed + reddit.  rmat (4.19 M nodes, 260 M nnz, F=256, K=3)
    needs ~35 GB of host memory and ~5 minutes."""
    which = sys.argv[1:] or ["tiny", "cora", "pubmed", "reddit"]
    if "tiny" in which:
        cases = tiny_cases()
        flat = {}
        for name, d in cases.items():
            for k, v in d.items():
                flat[f"{name}/{k}"] = v
        np.savez_compressed(os.path.join(HERE, "tiny_cases.npz"), **flat)
        print(f"tiny cases: {len(cases)}")
    which = [w for w in which if w != "tiny"]
    Ks = {"cora": (1, 2, 3), "pubmed": (1, 2), "reddit": (2,), "rmat": (3,)}
    out_json = os.path.join(HERE, "shapes.json")
    meta = json.load(open(out_json)) if os.path.exists(out_json) else {}
    rows_path = os.path.join(HERE, "shape_rows.npz")
    rows = dict(np.load(rows_path)) if os.path.exists(rows_path) else {}
    meta["_generator"] = {
        "reference": "bellaj09/SGC utils.py:23-30,92-97 + normalization.py:5-12, imported from "
                     + REF, "torch": torch.__version__, "numpy": np.__version__,
        "cpu_threads": torch.get_num_threads()}
    for shape in which:
        rec, samples = shape_case(shape, Ks[shape])
        meta[shape] = rec
        rows.update(samples)
    json.dump(meta, open(out_json, "w"), indent=1, sort_keys=True)
    np.savez_compressed(rows_path, **rows)


if __name__ == "__main__":
    main()
