"""Does a locality ordering of S pay at Reddit shape?  

    python scripts/locality_ab.py [--orders identity,rcm,degree,bfs] [--reps 10] [--only ORDER]

A symmetric permutation P S P^T that keeps every row's nonzero SEQUENCE (its
CSR storage order, i.e. the reference's FMA order) and only renames the
column ids gives bit-identical X_K rows (row i of the permuted result is row
perm[i] of the original).  This script builds that permuted CSR for several
orderings, checks the bit-identity on the GPU, and times the same product
propagation (sgc_amd.propagate, K = 2) on each, interleaved.  With --only it
runs one ordering's hops in a loop (for a rocprofv3 --pmc pass per order:
TCC_HIT / TCC_MISS give the L2 hit rate, FETCH_SIZE the bytes beyond L2).

Orderings: identity (the generator's random relabelling), rcm (reverse
Cuthill-McKee, scipy), degree (hubs first), bfs (breadth-first from the
largest hub: clusters neighbourhoods).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from sgc_amd import graphs  # noqa: E402
from sgc_amd.propagate import DeviceCSR, propagate  # noqa: E402


def ordering(S, name):
    n = S.n
    if name == "identity":
        return np.arange(n, dtype=np.int64)
    A = sp.csr_matrix((np.ones(S.nnz, np.float32), S.col_idx, S.row_ptr), shape=(n, n))
    if name == "rcm":
        from scipy.sparse.csgraph import reverse_cuthill_mckee
        return np.asarray(reverse_cuthill_mckee(A, symmetric_mode=True), dtype=np.int64)
    deg = np.diff(S.row_ptr)
    if name == "degree":
        return np.argsort(-deg, kind="stable").astype(np.int64)
    if name == "bfs":
        from scipy.sparse.csgraph import breadth_first_order
        order = breadth_first_order(A, int(np.argmax(deg)), directed=False,
                                    return_predecessors=False)
        seen = np.zeros(n, bool)
        seen[order] = True
        return np.concatenate([order, np.flatnonzero(~seen)]).astype(np.int64)
    raise ValueError(name)


def permuted(S, perm):
    """Rows in `perm` order (new row i = old row perm[i]), columns renamed by
    the inverse map, each row's nonzeros in their ORIGINAL storage order."""
    n = S.n
    inv = np.empty(n, np.int64)
    inv[perm] = np.arange(n)
    deg = np.diff(S.row_ptr).astype(np.int64)[perm]
    rp = np.zeros(n + 1, np.int64)
    np.cumsum(deg, out=rp[1:])
    starts = S.row_ptr[perm].astype(np.int64)
    idx = np.repeat(starts - rp[:-1], deg) + np.arange(rp[-1], dtype=np.int64)
    return rp.astype(np.int32), inv[S.col_idx[idx]].astype(np.int32), S.val[idx]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--orders", default="identity,rcm,degree,bfs")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default=None)
    ap.add_argument("--loops", type=int, default=20)
    args = ap.parse_args()
    S = graphs.synthetic_graph("reddit", seed=0)
    Xh = graphs.synthetic_features("reddit", S.n, 602, seed=1)
    dev = torch.device("cuda", 0)
    names = [args.only] if args.only else args.orders.split(",")
    runs = {}
    for nm in names:
        t0 = time.perf_counter()
        perm = ordering(S, nm)
        rp, ci, va = permuted(S, perm)
        t_order = time.perf_counter() - t0
        csr = DeviceCSR.from_host_arrays(rp, ci, va, device=dev)
        X = torch.from_numpy(np.ascontiguousarray(Xh[perm])).to(dev)
        out = torch.empty_like(X)
        propagate(csr, X, 2, out=out)  # plan + warm-up
        torch.cuda.synchronize()
        runs[nm] = (csr, X, out, perm, t_order)
    if args.only:
        csr, X, out, _, _ = runs[args.only]
        for _ in range(args.loops):
            propagate(csr, X, 2, out=out)
        torch.cuda.synchronize()
        print(json.dumps({"order": args.only, "loops": args.loops}))
        return
    ref = None
    ms = {nm: [] for nm in names}
    for _ in range(args.reps):
        for nm in names:  # interleaved A/B
            csr, X, out, _, _ = runs[nm]
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            propagate(csr, X, 2, out=out)
            e.record()
            torch.cuda.synchronize()
            ms[nm].append(s.elapsed_time(e))
    for nm in names:
        csr, X, out, perm, t_order = runs[nm]
        back = np.empty((S.n, 602), np.float32)
        back[perm] = out.cpu().numpy()
        if ref is None:
            ref = back
        same = bool(np.array_equal(back.view(np.uint32), ref.view(np.uint32)))
        print(json.dumps({"order": nm, "ms_per_step_median": float(np.median(ms[nm])),
                          "ms_per_step_min": float(np.min(ms[nm])),
                          "order_seconds": round(t_order, 2),
                          "bit_identical_to_identity": same}), flush=True)


if __name__ == "__main__":
    main()
