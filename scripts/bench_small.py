"""Small graphs (Cora / Pubmed shape, K=2): eager propagate() vs the same
hops replayed from a captured HIP graph (torch.cuda.CUDAGraph over the
library's launches on the capture stream, the hub side stream joined by
events; the replay includes copying X into the graph's static input).
One JSON line per case.

    python scripts/bench_small.py [--reps 200]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sgc_amd import graphs  # noqa: E402
from sgc_amd.propagate import DeviceCSR, GraphedPropagation, propagate  # noqa: E402


def timeit(fn, reps):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    args = ap.parse_args()
    for shape in ("cora", "pubmed"):
        spec = graphs.SHAPES[shape]
        S = graphs.synthetic_graph(shape, seed=0)
        X = torch.from_numpy(graphs.synthetic_features(shape, S.n, spec["features"], seed=1)).cuda()
        csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device="cuda")
        K = spec["hops"]
        out = torch.empty_like(X)
        eager = timeit(lambda: propagate(csr, X, K, out=out), args.reps)
        ref = out.clone()
        g = GraphedPropagation(csr, X.shape, K)
        g.run(X)
        torch.cuda.synchronize()
        assert torch.equal(g.out, ref), "graph replay differs from eager"
        graphed = timeit(lambda: g.run(X), args.reps)
        print(json.dumps({"shape": shape, "n": S.n, "nnz": S.nnz, "F": spec["features"], "K": K,
                          "eager_us": eager * 1e6, "graph_us": graphed * 1e6,
                          "eager_edges_per_s": K * S.nnz / eager,
                          "graph_edges_per_s": K * S.nnz / graphed}), flush=True)


if __name__ == "__main__":
    main()
