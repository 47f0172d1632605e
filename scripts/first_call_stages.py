"""Where the first sgc_precompute's extra time goes:
the stages of the public call, each synchronised, on a first adjacency and
then on a second adjacency object of the same graph (same process: only
per-process first-use costs differ), after the loaders' warm-up.

    python scripts/first_call_stages.py [--shape reddit] [--reserve-gb 0]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sgc_amd import graphs  # noqa: E402
from sgc_amd.propagate import column_groups_for, csr_of, propagate, warmup  # noqa: E402


def coo(S, dev):
    rows, cols, vals = S.coo()
    return torch.sparse_coo_tensor(torch.from_numpy(np.stack([rows, cols])),
                                   torch.from_numpy(vals), (S.n, S.n)).to(dev)


def stages(adj, X, K):
    rec = {}

    def mark(name, t0):
        torch.cuda.synchronize()
        rec[name] = round((time.perf_counter() - t0) * 1e3, 3)
        return time.perf_counter()
    t = time.perf_counter()
    csr = csr_of(adj)
    t = mark("ingest_ms", t)
    G = column_groups_for(csr, X.shape[1])
    parts = csr.column_groups(G) if G > 1 else [csr]
    t = mark("colsplit_ms", t)
    for c in parts:
        c.plan(0, csr.n_rows, None, None, X.shape[1])
    t = mark("plans_ms", t)
    out = torch.empty_like(X)
    t = mark("alloc_out_ms", t)
    propagate(csr, X, K, out=out)
    t = mark("propagate1_ms", t)
    propagate(csr, X, K, out=out)
    t = mark("propagate2_ms", t)
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="reddit")
    ap.add_argument("--reserve-gb", type=float, default=0.0)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    spec = graphs.SHAPES[args.shape]
    S = graphs.synthetic_graph(args.shape, seed=0)
    F, K = spec["features"], spec["hops"]
    X = torch.from_numpy(graphs.synthetic_features(args.shape, S.n, F, seed=1)).to(dev)
    a1, a2 = coo(S, dev), coo(S, dev)
    torch.cuda.synchronize()
    rec = {"shape": args.shape, "warmup_s": round(warmup(dev), 4), "reserve_gb": args.reserve_gb}
    if args.reserve_gb:
        b = torch.empty(int(args.reserve_gb * 2**30), dtype=torch.uint8, device=dev)
        del b
    rec["first_adjacency"] = stages(a1, X, K)
    rec["second_adjacency"] = stages(a2, X, K)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
