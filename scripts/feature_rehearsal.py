"""Rehearse the feature partition's per-rank step on ONE GPU.

    python scripts/feature_rehearsal.py [--shape reddit] [--P 2,4,8] [--align 4]

FeaturePartitionedPropagator needs no exchange between hops (column f of
X_{k+1} depends on column f of X_k only); its one exchange is the all-to-all
that turns the column blocks of X_K into row blocks (output="sharded", the
layout the row partition ends with).  Here each rank's exact step runs
through the propagator itself with that all-to-all replaced by a local copy
of the send buffer, so what is timed is the rank's compute (block copy,
K hops over all rows at the block's width, unpack of the P received blocks).
The all-to-all is then added at an assumed per-rank ingress bandwidth:
(P-1)/P of ceil(N/P) x B x 4 bytes per rank.  One JSON line per case.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sgc_amd import graphs  # noqa: E402
from sgc_amd.distributed import FeaturePartitionedPropagator, feature_bounds  # noqa: E402
from sgc_amd.propagate import DeviceCSR, propagate  # noqa: E402


class LocalFeaturePropagator(FeaturePartitionedPropagator):
    """The feature partition with the all-to-all replaced by a local copy."""

    def _all_to_all(self, recv, send):
        recv.copy_(send)
        return None


def timeit(fn, reps, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="reddit")
    ap.add_argument("--P", default="2,4,8")
    ap.add_argument("--align", type=int, default=4)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--bw", default="150,300,450", help="assumed all-to-all ingress GB/s per rank")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="schedule knob for sgc_set_tuning (results never depend on it)")
    args = ap.parse_args()
    if args.tune:
        from sgc_amd import _lib
        for kv in args.tune:
            k, v = kv.split("=")
            _lib.check(_lib.load().sgc_set_tuning(k.encode(), int(v)), f"set_tuning {kv}")
        print(json.dumps({"case": "tuning", "tune": args.tune}), flush=True)
    spec = graphs.SHAPES[args.shape]
    S = graphs.synthetic_graph(args.shape, seed=0)
    F, K, n = spec["features"], spec["hops"], S.n
    X0 = torch.from_numpy(graphs.synthetic_features(args.shape, n, F, seed=1)).cuda()
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device="cuda")
    out = torch.empty((n, F), device="cuda")
    t1 = timeit(lambda: propagate(csr, X0, K, out=out), args.reps)
    print(json.dumps({"case": "single", "shape": args.shape, "ms": t1}), flush=True)
    bws = [float(b) for b in args.bw.split(",")]
    for P in (int(p) for p in args.P.split(",")):
        fb, B = feature_bounds(F, P, args.align)
        Bn = -(-n // P)
        a2a = (P - 1) * Bn * B * 4  # bytes a rank receives
        ranks = []
        seen = {}
        for p in range(P):
            w = int(fb[p + 1] - fb[p])
            if w in seen:  # same block width, same work
                ranks.append(seen[w])
                continue
            prop = LocalFeaturePropagator(csr, rank=p, world_size=P, align=args.align)
            t = timeit(lambda: prop.propagate(X0, K, output="sharded"), args.reps)
            hop = timeit(lambda: prop.spmm_fn(X0[:, int(fb[p]):int(fb[p + 1])], 0, n,
                                              prop._buf("send", (P * Bn, B), X0)[:n, :w]),
                         args.reps)
            rec = {"case": "rank", "P": P, "rank": p, "cols": w, "compute_ms": t,
                   "one_hop_unaligned_ms": hop}
            print(json.dumps(rec), flush=True)
            seen[w] = rec
            ranks.append(rec)
            del prop
            torch.cuda.empty_cache()
        worst = max(r["compute_ms"] for r in ranks)
        proj = {f"{bw:g}GBps": worst + a2a / (bw * 1e9) * 1e3 for bw in bws}
        print(json.dumps({"case": "summary", "P": P, "block_floats": B, "single_ms": t1,
                          "max_rank_compute_ms": worst, "compute_only_speedup": t1 / worst,
                          "all_to_all_MB_per_rank": round(a2a / 1e6, 1),
                          "projected_step_ms": proj,
                          "projected_speedup": {k: t1 / v for k, v in proj.items()},
                          "assumption": "all-to-all not overlapped, at the given per-rank "
                                        "ingress GB/s; compute measured on one GPU per rank"}),
              flush=True)


if __name__ == "__main__":
    main()
