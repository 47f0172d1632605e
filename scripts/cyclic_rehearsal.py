"""Rehearse CyclicRowPropagator's P-rank step on ONE GPU, rank by rank.

    python scripts/cyclic_rehearsal.py [--shape reddit] [--P 8] [--groups 2,4,8] [--tiles 64]

For each (P, groups, tile) and each rank, the rank's exact launches (hop 1 in
G row chunks, later hops as G column-group passes chained by
SGC_SPMM_ACCUMULATE, the final pass of an exchanged hop in G row chunks) run
on this GPU through CyclicRowPropagator itself, with the all-gathers replaced
by nothing (the exchange buffers keep whatever they hold: kernel time does
not depend on the values).  Measured per rank: the compute-only wall time and
each launch's kernel time (sgc_timing_* hooks: light and hub kernel).

The exchange is modelled (the 8-GPU node is not available here): all-gather
c of a hop moves P * (local rows of group c) rows x Fp floats, a rank
receiving (P-1)/P of it at an assumed per-rank ingress bandwidth, on one comm
stream, starting when row chunk c is done; pass g of the next hop starts when
all-gather g has arrived and the previous launch is done.  Projected step =
measured compute-only time + (model at bandwidth - model with a free
exchange), for the slowest rank; speed-up against the measured single-GPU
step.  Same method as scripts/p8_rehearsal.py for the contiguous row blocks.
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
from sgc_amd.distributed import CyclicRowPropagator  # noqa: E402
from sgc_amd.propagate import (DeviceCSR, aligned_ld, collect_kernel_timing,  # noqa: E402
                               kernel_timing, propagate)


class LocalCyclic(CyclicRowPropagator):
    """Compute-only: the exchange is skipped."""

    def _all_gather(self, full, loc):
        # no copy (the exchange is modelled), but the consumer still waits for
        # the work enqueued on the comm stream so far, as RCCL's wait() would
        from sgc_amd.distributed import _StreamDone
        return _StreamDone(torch.cuda.current_stream(full.device)) if full.is_cuda else None


def timeit(fn, reps=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def launch_plan(K, G, output="sharded"):
    """[(hop, kind, index)] in issue order, as CyclicRowPropagator.propagate
    enqueues them: kind "chunk" = a row chunk of an exchanged hop's final
    pass (its all-gather follows), "pass" = a column-group pass over all rows."""
    plan = []
    for h in range(K):
        exchanged = h < K - 1 or output == "replicated"
        passes = 1 if h == 0 else G
        for p in range(passes):
            g = None if h == 0 else p
            if p == passes - 1 and exchanged:
                plan += [(h, "chunk", c, g) for c in range(G)]
            else:
                plan.append((h, "pass", p, g))
    return plan


def durations(plan, light, hub, has_hub):
    """(main-stream ms, hub-stream ms) per plan entry from the timing records.
    Hop 1's chunks are split launches: first the hub-only launches of all
    chunks (a record each, empty light interval, hub time set -- none for a
    chunk without hub rows), then the light launches (hub None).  Every other
    launch is one record whose hub kernel is joined, so its duration is the
    longer of the two."""
    recs = list(zip(light, hub))
    out, i = [], 0
    n0 = sum(1 for p in plan if p[0] == 0 and p[1] == "chunk")
    hubs = []
    while i < len(recs) and len(hubs) < n0 and recs[i][1] is not None and recs[i][0] < 0.02:
        hubs.append(recs[i][1])
        i += 1
    for h, kind, idx, g in plan:
        lt, hb = recs[i]
        i += 1
        if h == 0 and kind == "chunk":
            out.append((lt, 0.0))
        else:
            out.append((max(lt, hb or 0.0), 0.0))
    # the hub-only launches run back to back on the hub stream from the start
    # of hop 1; chunks without hub rows (has_hub False) have no record
    owners = [c for c in range(n0) if has_hub[c]]
    if len(owners) != len(hubs):
        raise RuntimeError(f"{len(hubs)} hub records for {len(owners)} chunks with hub rows")
    for c, hb in zip(owners, hubs):
        out[c] = (out[c][0], hb)
    if i != len(recs):
        raise RuntimeError(f"{len(recs)} timing records, {i} matched to the launch plan: {recs}")
    return out


def simulate(plan, dur, G, bytes_per_gather, P, bw_gbs):
    """One rank's timeline (ms): dur[i] = (main, hub-stream) ms of launch i."""
    main = comm = hub_t = 0.0
    arrive_prev = [0.0] * G   # all-gathers of the previous exchanged hop
    arrive_cur = []
    hop = 0
    for i, (h, kind, idx, g) in enumerate(plan):
        if h != hop:
            arrive_prev, arrive_cur, hop = arrive_cur, [], h
        start = main
        if g is not None and kind == "pass":
            start = max(start, arrive_prev[g])
        if g is not None and kind == "chunk":  # final pass g = G-1 needs gather G-1
            start = max(start, arrive_prev[G - 1])
        d_main, d_hub = dur[i]
        hub_t = hub_t + d_hub  # hop-1 hub launches: back to back from t = 0
        main = start + d_main
        if kind == "chunk":
            t = (P - 1) / P * bytes_per_gather / (bw_gbs * 1e9) * 1e3
            comm = max(comm, main, hub_t) + t
            arrive_cur.append(comm)
    return max(main, hub_t)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="reddit")
    ap.add_argument("--P", default="8", help="comma list of rank counts")
    ap.add_argument("--groups", default="2,4,8")
    ap.add_argument("--tiles", default="64")
    ap.add_argument("--bw", default="300,450,600", help="assumed all-gather ingress GB/s per rank")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--ranks", default="all", help="'all' or a comma list of ranks to time")
    ap.add_argument("--pad-input", default="auto", choices=["auto", "yes", "no"],
                    help="re-lay X_0 into 128-B rows before hop 1 (auto: P <= 4)")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="sgc_set_tuning knob (applies to every launch, single-GPU step included)")
    args = ap.parse_args()
    if args.tune:
        from sgc_amd import _lib
        for kv in args.tune:
            k, v = kv.split("=", 1)
            _lib.check(_lib.load().sgc_set_tuning(k.encode(), int(v)), f"set_tuning {kv}")
    spec = graphs.SHAPES[args.shape]
    S = graphs.synthetic_graph(args.shape, seed=0)
    F, K, n = spec["features"], spec["hops"], S.n
    Fp = aligned_ld(F)
    X0 = torch.from_numpy(graphs.synthetic_features(args.shape, n, F, seed=1)).cuda()
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device="cuda")
    out = torch.empty((n, F), device="cuda")
    t1 = timeit(lambda: propagate(csr, X0, K, out=out), args.reps)
    del csr
    print(json.dumps({"case": "single", "shape": args.shape, "ms": t1 * 1e3, "tune": args.tune}),
          flush=True)
    bws = [float(b) for b in args.bw.split(",")]
    for P in (int(x) for x in args.P.split(",")):
        for tile in (int(x) for x in args.tiles.split(",")):
            for G in (int(x) for x in args.groups.split(",")):
                ranks = range(P) if args.ranks == "all" else [int(r) for r in args.ranks.split(",")]
                recs = []
                for r in ranks:
                    cp = LocalCyclic(S.row_ptr, S.col_idx, S.val, r, P, "cuda", tile=tile,
                                     groups=G, pad_input={"auto": None, "yes": True,
                                                          "no": False}[args.pad_input])
                    sh = cp.shard
                    t = timeit(lambda: cp.propagate(X0, K, output="sharded"), args.reps)
                    torch.cuda.synchronize()
                    collect_kernel_timing()
                    kernel_timing(True)
                    cp.propagate(X0, K, output="sharded")
                    kernel_timing(False)
                    light, hub = collect_kernel_timing()
                    plan = launch_plan(K, G)
                    ci = sh.csr_input
                    th, hb = cp._th  # the rank-level thresholds every launch used
                    pad = P <= 4 if args.pad_input == "auto" else args.pad_input == "yes"
                    has_hub = [ci.plan(c * sh.group_rows, (c + 1) * sh.group_rows, th, hb,
                                       Fp if pad else F).n_hub > 0  # hop-1 width
                               for c in range(G)]
                    dur = durations(plan, light, hub, has_hub)
                    gbytes = P * sh.group_rows * Fp * 4
                    free = simulate(plan, dur, G, gbytes, P, 1e12)
                    proj = {f"{bw:g}GBps": t * 1e3 + simulate(plan, dur, G, gbytes, P, bw) - free
                            for bw in bws}
                    rec = {"case": "rank", "P": P, "tile": tile, "groups": G, "rank": r,
                           "rows": sh.n_valid, "nnz": sh.nnz, "compute_ms": t * 1e3,
                           "kernel_ms_sum": sum(d for d, _ in dur),
                           "launch_ms": [[round(a, 4), round(b, 4)] for a, b in dur],
                           "proj_ms": proj}
                    recs.append(rec)
                    print(json.dumps(rec), flush=True)
                    del cp
                    torch.cuda.empty_cache()
                worst = max(x["compute_ms"] for x in recs)
                pj = {k: max(x["proj_ms"][k] for x in recs) for k in recs[0]["proj_ms"]}
                ex = (P - 1) / P * P * recs[0]["rows"] * Fp * 4 * (K - 1)
                print(json.dumps({"case": "summary", "P": P, "tile": tile, "groups": G,
                                  "single_ms": t1 * 1e3, "max_rank_compute_ms": worst,
                                  "compute_only_speedup": t1 * 1e3 / worst,
                                  "nnz_max_over_mean": max(x["nnz"] for x in recs) /
                                  np.mean([x["nnz"] for x in recs]),
                                  "exchange_MB_per_rank": round(ex / 1e6, 1),
                                  "projected_step_ms": pj,
                                  "projected_speedup": {k: t1 * 1e3 / v for k, v in pj.items()},
                                  "assumption": "G all-gathers per exchanged hop at the given "
                                                "per-rank ingress GB/s on one comm stream; "
                                                "kernel times measured on one GPU per rank"}),
                      flush=True)


if __name__ == "__main__":
    main()
