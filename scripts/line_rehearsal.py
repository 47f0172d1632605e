"""Rehearse the line partition's per-rank step on ONE GPU.

    python scripts/line_rehearsal.py [--shape reddit] [--P 2,4,8] [--link-gbps 57.6]

LinePartitionedPropagator: rank p owns whole 128-B lines of features over all
rows (no exchange between hops) plus an nnz-balanced row block of the tail
features, whose rows are all-gathered after every hop.  Each rank's exact step
runs through the propagator itself with the collectives replaced by local
copies (the gather copies the rank's own block into its slot; the other
ranks' slots hold zeros), so what is timed is the rank's compute: block
copies, the K main hops over all rows, the K tail hops over its rows, the
last hop's unpack.  The exchanges are then modelled at a stated link rate (one
xGMI link per GPU pair, --link-gbps each way, a rank's ingress (P-1) links):
  * each hop's tail gather rides under that hop's main launch (the tail
    launch and its gather run on the tail stream beside it; the model adds
    whatever the main hop does not cover);
  * sharded output: the main blocks' all-to-all ((P-1)/P of the rank's rows x
    W floats) after the last hop;
  * replicated output (the public sgc_precompute): every rank receives
    (P-1)/P of X_K -- modelled as after the last hop, no overlap credited.
One JSON line per rank and a summary per P.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sgc_amd import graphs  # noqa: E402
from sgc_amd.distributed import (LinePartitionedPropagator, equal_row_bounds,  # noqa: E402
                                 line_bounds, make_shard)
from sgc_amd.propagate import SPMM_X_PADDED, SPMM_Y_PADDED, DeviceCSR, propagate  # noqa: E402


class LocalLinePropagator(LinePartitionedPropagator):
    """The line partition with the collectives replaced by local copies."""

    def _buf(self, key, shape, like):
        b = self._bufs.get(key)
        if b is None or tuple(b.shape) != tuple(shape) or b.device != like.device:
            b = torch.zeros(shape, dtype=torch.float32, device=like.device)
            self._bufs[key] = b
        return b

    def _collective(self, kind, dst, src):
        if kind == "gather":
            m = src.shape[0]
            dst[self.rank * m:(self.rank + 1) * m].copy_(src)
        else:
            m = min(src.shape[0], dst.shape[0])
            dst[:m].copy_(src[:m])
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
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--ranks", default="all", help="all, or a comma list of ranks to time")
    ap.add_argument("--link-gbps", type=float, default=57.6,
                    help="per-peer xGMI rate each way (one link per GPU pair): a rank's "
                         "ingress is (P-1) x this")
    args = ap.parse_args()
    spec = graphs.SHAPES[args.shape]
    S = graphs.synthetic_graph(args.shape, seed=0)
    F, K, n = spec["features"], spec["hops"], S.n
    X0 = torch.from_numpy(graphs.synthetic_features(args.shape, n, F, seed=1)).cuda()
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device="cuda")
    out = torch.empty((n, F), device="cuda")
    t1 = timeit(lambda: propagate(csr, X0, K, out=out), args.reps)
    print(json.dumps({"case": "single", "shape": args.shape, "ms": t1}), flush=True)
    for P in (int(p) for p in args.P.split(",")):
        W, T = line_bounds(F, P)
        wt = F - T
        ldt = (max(wt, 1) + 31) // 32 * 32
        ingress = (P - 1) * args.link_gbps * 1e9
        Bn = -(-n // P)
        ranks = []
        sel = range(P) if args.ranks == "all" else [int(r) for r in args.ranks.split(",")]
        for p in sel:
            shard = make_shard(S.row_ptr, S.col_idx, S.val, p, P, "cuda")
            prop = LocalLinePropagator(shard, csr=csr)
            t_rep = timeit(lambda: prop.propagate(X0, K, output="replicated"), args.reps)
            t_sh = timeit(lambda: prop.propagate(X0, K, output="sharded"), args.reps)
            # one main hop and one tail hop in the propagator's own buffers
            w = min((p + 1) * W, F) - min(p * W, F)
            ld = (max(W, 1) + 31) // 32 * 32
            t_main = t_tail = 0.0
            if w:
                Xm = prop._buf(("h", 1), (n, ld), X0)[:, :w]
                Ym = prop._buf("send", (P * Bn, max(W, 1)), X0)[:n, :w]
                t_main = timeit(lambda: prop.main_spmm_fn(Xm, 0, n, Ym,
                                                          flags=SPMM_X_PADDED | SPMM_Y_PADDED),
                                args.reps)
            if wt and shard.rows:
                full = prop._buf(("tf", 1), (P * shard.block, ldt), X0)
                loc = prop._buf(("tl", 0), (shard.block, ldt), X0)
                wt4 = min(ldt, (wt + 3) // 4 * 4)
                t_tail = timeit(lambda: prop.tail_spmm_fn(shard, full[:, :wt4],
                                                          loc[:shard.rows, :wt4], "gathered"),
                                args.reps)
            gather_b = (P - 1) * shard.block * ldt * 4
            t_gather = gather_b / ingress * 1e3
            # exposed part of each tail gather: what the main hop running
            # beside it (the same hop's, on the main stream) does not cover
            exposed = K * max(0.0, t_gather - t_main)
            a2a_b = (P - 1) * Bn * max(W, 1) * 4
            sharded = t_sh + exposed + (a2a_b / ingress * 1e3)
            rep_b = (P - 1) / P * n * F * 4
            replicated = t_rep + exposed + rep_b / ingress * 1e3
            rec = {"case": "rank", "P": P, "rank": p, "main_floats": w, "tail_floats": wt,
                   "tail_rows": shard.rows, "tail_block_rows": shard.block,
                   "compute_sharded_ms": t_sh, "compute_replicated_ms": t_rep,
                   "main_hop_ms": t_main, "tail_hop_ms": t_tail,
                   "tail_gather_MB": round(gather_b / 1e6, 1), "tail_gather_ms": t_gather,
                   "projected_sharded_ms": sharded, "projected_replicated_ms": replicated}
            print(json.dumps(rec), flush=True)
            ranks.append(rec)
            del prop, shard
            torch.cuda.empty_cache()
        worst = max(r["compute_sharded_ms"] for r in ranks)
        ps = max(r["projected_sharded_ms"] for r in ranks)
        pr = max(r["projected_replicated_ms"] for r in ranks)
        print(json.dumps({"case": "summary", "P": P, "main_floats": W, "tail_floats": wt,
                          "single_ms": t1, "max_rank_compute_ms": worst,
                          "compute_only_speedup": t1 / worst,
                          "projected_sharded_ms": ps, "projected_sharded_speedup": t1 / ps,
                          "projected_replicated_ms": pr,
                          "projected_replicated_speedup": t1 / pr,
                          "link_GBps_each_way": args.link_gbps,
                          "assumption": "one xGMI link per GPU pair at link_GBps each way; "
                                        "compute measured on one GPU per rank; each tail "
                                        "gather under its hop's main launch; the main "
                                        "blocks' exchange after the last hop"}), flush=True)


if __name__ == "__main__":
    main()
