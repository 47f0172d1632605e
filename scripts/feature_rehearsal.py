"""Rehearse the feature partition's per-rank step on ONE GPU.

    python scripts/feature_rehearsal.py [--shape reddit] [--P 2,4,8] [--align 4]
                                        [--exchange alltoall,pairwise] [--link-gbps 57.6]

FeaturePartitionedPropagator needs no exchange between hops (column f of
X_{k+1} depends on column f of X_k only); its one exchange is the all-to-all
that turns the column blocks of X_K into row blocks (output="sharded", the
layout the row partition ends with).  Here each rank's exact step runs
through the propagator itself with that all-to-all replaced by a local copy
of the send buffer, so what is timed is the rank's compute (block copy,
K hops over all rows at the block's width, unpack of the P received blocks).
The exchange is then modelled at a stated link rate: one xGMI link per GPU
pair, --link-gbps each way, so a rank's ingress is (P-1) links; the
all-to-all ((P-1)/P of ceil(N/P) x B x 4 bytes per rank) after the last hop,
the pairwise exchange overlapped with it on a timeline (pairwise_projection).
One JSON line per case.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sgc_amd import graphs  # noqa: E402
from sgc_amd.distributed import FeaturePartitionedPropagator, _copy_cols, feature_bounds  # noqa: E402
from sgc_amd.propagate import SPMM_X_PADDED, SPMM_Y_PADDED, DeviceCSR, propagate  # noqa: E402


class LocalFeaturePropagator(FeaturePartitionedPropagator):
    """The feature partition with the exchange replaced by local copies."""

    def _all_to_all(self, recv, send):
        recv.copy_(send)
        return None

    def _exchange_pair(self, send, dst, recv, src):
        m = min(send.shape[0], recv.shape[0])
        if m:
            recv[:m].copy_(send[:m])
        return []


def pairwise_projection(t_c, t_hop, t_unpack, P, k, piece_bytes, link_gbps):
    """Step time of the pairwise exchange: hop K starts at t0 = t_c - t_hop -
    t_unpack and computes the P-1 destination blocks in k pieces each, then
    the rank's own block (equal time per row); piece i of destination j is
    sent when computed, on the link to that peer (one link per GPU pair,
    full duplex: a rank's sends to different peers run in parallel, pieces to
    one peer in sequence); the unpack waits for the last receive."""
    t0 = t_c - t_hop - t_unpack
    dt = t_hop / (P * k)
    lt = piece_bytes / (link_gbps * 1e9) * 1e3
    end = 0.0
    for j in range(P - 1):
        free = 0.0
        for i in range(k):
            ready = t0 + (j * k + i + 1) * dt
            free = max(free, ready) + lt
        end = max(end, free)
    return max(t_c, end + t_unpack)


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
    ap.add_argument("--link-gbps", type=float, default=57.6,
                    help="per-peer xGMI rate each way (one link per GPU pair): a rank's "
                         "ingress is (P-1) x this")
    ap.add_argument("--exchange", default="alltoall,pairwise")
    ap.add_argument("--pieces", type=int, default=None, help="pairwise: row pieces per destination")
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
    for P in (int(p) for p in args.P.split(",")):
        fb, B = feature_bounds(F, P, args.align)
        Bn = -(-n // P)
        a2a = (P - 1) * Bn * B * 4  # bytes a rank receives
        ingress = (P - 1) * args.link_gbps
        for mode in args.exchange.split(","):
            ranks = []
            seen = {}
            for p in range(P):
                w = int(fb[p + 1] - fb[p])
                if w in seen:  # same block width, same work
                    ranks.append(seen[w])
                    continue
                prop = LocalFeaturePropagator(csr, rank=p, world_size=P, align=args.align,
                                              exchange=mode, pieces=args.pieces)
                t = timeit(lambda: prop.propagate(X0, K, output="sharded"), args.reps)
                ld = (B + 31) // 32 * 32
                Xw = prop._buf(("h", 0), (n, ld), X0)[:, :w]
                Yw = prop._buf("send", (P * Bn, B), X0)[:n, :w]
                hop = timeit(lambda: prop.spmm_fn(Xw, 0, n, Yw, flags=SPMM_X_PADDED | SPMM_Y_PADDED),
                             args.reps)
                rows = int(min(n, (p + 1) * Bn) - min(n, p * Bn))
                outb = torch.empty((rows, F), device="cuda")
                recv = prop._buf("recv", (P * Bn, B), X0)

                def unpack():
                    for q in range(P):
                        q0, q1 = int(fb[q]), int(fb[q + 1])
                        if q != p and q1 > q0 and rows:
                            _copy_cols(recv[q * Bn:q * Bn + rows, :q1 - q0], outb[:, q0:q1])
                t_unpack = timeit(unpack, args.reps)
                rec = {"case": "rank", "P": P, "exchange": mode, "rank": p, "cols": w,
                       "compute_ms": t, "hop_ms": hop, "unpack_ms": t_unpack,
                       "pieces": prop._pieces(P)}
                if mode == "pairwise":
                    k = prop._pieces(P)
                    rec["projected_ms"] = pairwise_projection(t, hop, t_unpack, P, k,
                                                              Bn * B * 4 / k, args.link_gbps)
                else:
                    rec["projected_ms"] = t + a2a / (ingress * 1e9) * 1e3
                print(json.dumps(rec), flush=True)
                seen[w] = rec
                ranks.append(rec)
                del prop
                torch.cuda.empty_cache()
            worst = max(r["compute_ms"] for r in ranks)
            proj = max(r["projected_ms"] for r in ranks)
            print(json.dumps({"case": "summary", "P": P, "exchange": mode, "block_floats": B,
                              "single_ms": t1, "max_rank_compute_ms": worst,
                              "compute_only_speedup": t1 / worst,
                              "exchange_MB_per_rank": round(a2a / 1e6, 1),
                              "link_GBps_each_way": args.link_gbps,
                              "ingress_GBps": ingress, "projected_step_ms": proj,
                              "projected_speedup": t1 / proj,
                              "assumption": "one xGMI link per GPU pair at link_GBps each way; "
                                            "compute measured on one GPU per rank; pairwise: "
                                            "sends overlapped with the last hop (timeline model), "
                                            "alltoall: after it"}), flush=True)


if __name__ == "__main__":
    main()
