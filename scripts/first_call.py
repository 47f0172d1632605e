"""Where the first sgc_precompute call's time goes (a fresh process).

    python scripts/first_call.py [--shape reddit]

reddit.py calls sgc_precompute once (reference reddit.py:43), so the first
call is the one a user sees.  Printed, in order, all with synchronised
timers: the first call on a tiny graph (loads the library's code objects,
first allocations), the first call on the shape's graph (ingest, plan,
buffers, hops), a second call on the same adjacency (steady state), and the
first call on a new adjacency object of the same graph (ingest + plan with
the buffers already in torch's cache).  Then the ingest and plan alone.
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
from sgc_amd.utils import sgc_precompute  # noqa: E402


def coo(S, dev):
    rows, cols, vals = S.coo()
    return torch.sparse_coo_tensor(torch.from_numpy(np.stack([rows, cols])),
                                   torch.from_numpy(vals), (S.n, S.n)).to(dev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="reddit")
    ap.add_argument("--stages", action="store_true", help="time the tiny call's stages first")
    ap.add_argument("--warm", action="store_true",
                    help="call propagate.warmup() first (what the drop-in loaders do)")
    ap.add_argument("--reserve-gb", type=float, default=0.0,
                    help="allocate and free this many GiB first (held in torch's cache)")
    ap.add_argument("--no-tiny", action="store_true",
                    help="skip the tiny call: first_call_s is the process's first call")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    spec = graphs.SHAPES[args.shape]
    T = graphs.synthetic_graph("cora", seed=1, n=500, edges=2000)
    S = graphs.synthetic_graph(args.shape, seed=0)
    F, K = spec["features"], spec["hops"]
    X = torch.from_numpy(graphs.synthetic_features(args.shape, S.n, F, seed=1)).to(dev)
    Xt = torch.from_numpy(graphs.synthetic_features("cora", T.n, F, seed=1)).to(dev)
    at, a1, a2 = coo(T, dev), coo(S, dev), coo(S, dev)
    torch.cuda.synchronize()
    rec = {"shape": args.shape, "warm": args.warm, "tiny": not args.no_tiny,
           "reserve_gb": args.reserve_gb}
    if args.reserve_gb > 0:
        t = time.perf_counter()
        blk = torch.empty(int(args.reserve_gb * 2**30), dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        del blk
        rec["reserve_s"] = round(time.perf_counter() - t, 4)
    if args.warm:
        from sgc_amd.propagate import warmup
        rec["warmup_s"] = round(warmup(dev), 4)
    if args.stages:  # the tiny first call's stages, each first in the process
        from sgc_amd.propagate import DeviceCSR, propagate
        t = time.perf_counter()
        c = DeviceCSR.from_torch(coo(T, dev))
        torch.cuda.synchronize()
        rec["stage_ingest_s"] = round(time.perf_counter() - t, 4)
        t = time.perf_counter()
        c.plan(0, T.n, None, None, F)
        torch.cuda.synchronize()
        rec["stage_plan_s"] = round(time.perf_counter() - t, 4)
        t = time.perf_counter()
        propagate(c, Xt, K)
        torch.cuda.synchronize()
        rec["stage_propagate_s"] = round(time.perf_counter() - t, 4)
    if not args.no_tiny:
        t = time.perf_counter()
        _, s = sgc_precompute(Xt, at, K)
        rec["tiny_first_call_s"] = round(time.perf_counter() - t, 4)
        rec["tiny_first_call_reported_s"] = round(s, 4)
    for key, adj in (("first_call_s", a1), ("second_call_s", a1), ("new_adj_first_call_s", a2),
                     ("new_adj_second_call_s", a2)):
        _, s = sgc_precompute(X, adj, K)
        rec[key] = round(s, 4)
    csr = a2._sgc_amd_csr[1]
    rec["ingest_s"] = round(csr.ingest_seconds, 4)
    from sgc_amd.propagate import DeviceCSR
    c = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device=dev)
    torch.cuda.synchronize()
    t = time.perf_counter()
    c.plan(0, S.n, None, None, F)
    torch.cuda.synchronize()
    rec["plan_s"] = round(time.perf_counter() - t, 4)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
