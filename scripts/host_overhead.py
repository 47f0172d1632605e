"""Host-side cost of one public sgc_precompute call on the small shapes.

    python scripts/host_overhead.py [--shapes cora,pubmed] [--reps 200]

The Cora / Pubmed hops take 20-50 us on the GPU, so the call's fixed host
costs decide their edges/s.  Prints, per shape (medians over reps): the whole
synchronised call; torch.cuda.synchronize() on an idle device; propagate()'s
host time to enqueue everything (no wait); the hops' GPU time (events); and
the same call under a HIP graph replay for comparison.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from sgc_amd import graphs  # noqa: E402
from sgc_amd.propagate import propagate  # noqa: E402
from sgc_amd.utils import sgc_precompute  # noqa: E402


def med(f, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="cora,pubmed")
    ap.add_argument("--reps", type=int, default=200)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    for shape in args.shapes.split(","):
        spec = graphs.SHAPES[shape]
        S = graphs.synthetic_graph(shape, seed=0)
        X = torch.from_numpy(graphs.synthetic_features(shape, S.n, spec["features"],
                                                       seed=1)).to(dev)
        r, c, v = S.coo()
        adj = torch.sparse_coo_tensor(torch.from_numpy(np.stack([r, c])), torch.from_numpy(v),
                                      (S.n, S.n)).to(dev)
        K = spec["hops"]
        sgc_precompute(X, adj, K)
        csr = adj._sgc_amd_csr[1]
        torch.cuda.synchronize()
        rec = {"shape": shape}
        rec["call_us"] = med(lambda: sgc_precompute(X, adj, K), args.reps)
        rec["sync_idle_us"] = med(torch.cuda.synchronize, args.reps)
        out = torch.empty_like(X)

        def enqueue():
            propagate(csr, X, K, out=out)
        enqueue()
        torch.cuda.synchronize()
        rec["propagate_enqueue_us"] = med(enqueue, min(args.reps, 100))
        torch.cuda.synchronize()
        ev = []
        for _ in range(50):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            propagate(csr, X, K, out=out)
            e.record()
            ev.append((s, e))
        torch.cuda.synchronize()
        rec["gpu_events_us"] = float(np.median([s.elapsed_time(e) for s, e in ev])) * 1e3
        from sgc_amd.propagate import GraphedPropagation
        g = GraphedPropagation(csr, tuple(X.shape), K)
        g.run(X)
        torch.cuda.synchronize()
        rec["graph_replay_call_us"] = med(lambda: (g.run(X), torch.cuda.synchronize()),
                                          args.reps)
        print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v)
                          for k, v in rec.items()}), flush=True)


if __name__ == "__main__":
    main()
