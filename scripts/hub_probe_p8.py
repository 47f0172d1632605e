"""Hub rows of one P = 8 rank: the HUB_ONLY launch alone, the light launch
alone, and both together (as hop 1 of the cyclic pipeline runs them), with
the hub-row statistics of the rank's plan.

    python scripts/hub_probe_p8.py [--P 8] [--rank 0] [--hub-threshold N]
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
from sgc_amd.distributed import CyclicRowPropagator, _cyclic_spmm  # noqa: E402


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--hub-threshold", type=int, default=None)
    ap.add_argument("--heavy-threshold", type=int, default=None)
    ap.add_argument("--groups", type=int, default=1)
    args = ap.parse_args()
    S = graphs.synthetic_graph("reddit", seed=0)
    F = 602
    X0 = torch.from_numpy(graphs.synthetic_features("reddit", S.n, F, seed=1)).cuda()
    cp = CyclicRowPropagator(S.row_ptr, S.col_idx, S.val, args.rank, args.P, "cuda",
                             groups=args.groups)
    sh = cp.shard
    th, hub = cp._thresholds(F)
    if args.hub_threshold:
        hub = args.hub_threshold
    if args.heavy_threshold:
        th = args.heavy_threshold
    csr = sh.csr_input
    R = sh.rows
    out = torch.empty((R, F), device="cuda")
    pl = csr.plan(0, R, th, hub, F)
    rp = csr.row_ptr.cpu().numpy().astype(np.int64)
    deg = np.diff(rp)
    hubs = np.sort(deg[deg > hub])[::-1]
    rec = {"P": args.P, "rank": args.rank, "heavy_rows": int(pl.n_heavy - pl.n_hub), "heavy_threshold": th, "hub_threshold": hub,
           "n_hub": int(pl.n_hub), "hub_nnz": int(hubs.sum()), "rank_nnz": sh.nnz,
           "hub_degrees_top": hubs[:8].tolist(), "max_hub_degree": pl.max_hub_degree}
    th_t = (th, hub)
    rec["hub_alone_ms"] = timeit(lambda: _cyclic_spmm(csr, X0, out, (0, R), False, "hub", th_t))
    rec["light_alone_ms"] = timeit(lambda: _cyclic_spmm(csr, X0, out, (0, R), False, "light",
                                                        th_t))
    rec["joined_ms"] = timeit(lambda: _cyclic_spmm(csr, X0, out, (0, R), False, "all", th_t))
    side = torch.cuda.Stream()

    def both():
        ev = torch.cuda.Event()
        ev.record()
        side.wait_event(ev)
        with torch.cuda.stream(side):
            _cyclic_spmm(csr, X0, out, (0, R), False, "hub", th_t)
        _cyclic_spmm(csr, X0, out, (0, R), False, "light", th_t)
        torch.cuda.current_stream().wait_stream(side)
    rec["hub_first_concurrent_ms"] = timeit(both)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
