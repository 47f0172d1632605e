"""Upper bound for an LDS-resident hot-row table in the light kernel.

    python scripts/hot_bound.py [--shape reddit] [--hot 0,64,120,256,512]

Timing only (the results are NOT the reference's): the nonzeros whose column
is one of the H most frequent columns are pointed at the single hottest
column, so their gathers hit one X row that every CU keeps in its L1/L2 --
what serving them from LDS would at best save -- and the L2 holds the next
hottest rows instead.  One K-hop propagate per H, interleaved rounds.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sgc_amd import graphs  # noqa: E402
from sgc_amd.propagate import DeviceCSR, propagate  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="reddit")
    ap.add_argument("--hot", default="0,64,120,256,512")
    ap.add_argument("--rounds", type=int, default=8)
    args = ap.parse_args()
    S = graphs.synthetic_graph(args.shape, seed=0)
    F, K = graphs.SHAPES[args.shape]["features"], graphs.SHAPES[args.shape]["hops"]
    X = torch.from_numpy(graphs.synthetic_features(args.shape, S.n, F, seed=1)).cuda()
    cnt = np.bincount(S.col_idx, minlength=S.n)
    order = np.argsort(-cnt, kind="stable")
    csrs = {}
    for H in (int(h) for h in args.hot.split(",")):
        col = S.col_idx.copy()
        if H > 0:
            hot = np.zeros(S.n, bool)
            hot[order[:H]] = True
            col[hot[col]] = order[0]
        csrs[H] = DeviceCSR.from_host_arrays(S.row_ptr, col, S.val, device="cuda")
        share = float(cnt[order[:H]].sum()) / S.nnz if H else 0.0
        print(json.dumps({"case": "hot", "H": H, "nnz_share": round(share, 4)}), flush=True)
    out = torch.empty_like(X)
    ms = {H: [] for H in csrs}
    for H, c in csrs.items():
        propagate(c, X, K, out=out)
    torch.cuda.synchronize()
    for _ in range(args.rounds):
        for H, c in csrs.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            propagate(c, X, K, out=out)
            e.record()
            torch.cuda.synchronize()
            ms[H].append(s.elapsed_time(e))
    for H in csrs:
        print(json.dumps({"case": "time", "shape": args.shape, "K": K, "H": H,
                          "median_ms": round(float(np.median(ms[H])), 4),
                          "min_ms": round(float(np.min(ms[H])), 4)}), flush=True)


if __name__ == "__main__":
    main()
