"""Rehearse the row-partitioned step of P ranks on ONE GPU, rank by rank.

    python scripts/p8_rehearsal.py [--shape reddit] [--layouts 8x1,4x2] [--group-floats 224]

For each layout R x C (R nnz-balanced row blocks x C feature blocks, P = R*C;
C = 1 is the row partition, C > 1 sgc_amd.distributed.TiledPropagator) and
each rank, the rank's exact work runs on this GPU through
RowPartitionedPropagator itself (nnz-balanced blocks, split hub/light
launches on their streams, feature groups) with the all-gather replaced by
a local copy of the rank's own block into the exchange buffer: what remains
is the rank's compute, with the same launch sequence and stream overlap as
on the node.  Per rank it prints the compute-only step time and the per-group
light / hub kernel times (sgc_timing_* hooks).

The exchange is then modelled (it needs the 8-GPU node) and ADDED to the
rank's measured compute-only time as far as the model leaves it exposed: each
hop that feeds
another all-gathers group g (P*B rows x group width x 4 B; a rank receives
(P-1)/P of it) on one comm stream at an assumed per-rank ingress bandwidth,
starting when group g's light and hub kernels are done and the previous
group's gather has finished; group g of the next hop starts when its gather
has arrived and the previous group's light kernel is done.  The projected
step is the slowest rank's timeline; the speed-up is against the measured
single-GPU step.  Assumptions are printed with the numbers.
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
from sgc_amd.distributed import (RowPartitionedPropagator, equal_row_bounds,  # noqa: E402
                                 feature_bounds, make_shard, nnz_balanced_bounds)
from sgc_amd.propagate import (DeviceCSR, collect_kernel_timing, kernel_timing,  # noqa: E402
                               propagate)


class LocalRowPropagator(RowPartitionedPropagator):
    """The row partition with the all-gather replaced by a local copy of this
    rank's block (compute-only rehearsal on one GPU)."""

    def _all_gather(self, full, loc):
        # the copy runs on the current (comm) stream: hand back a handle whose
        # wait() orders the consumer after it, like RCCL's work object
        from sgc_amd.distributed import _StreamDone
        s = self.shard
        full[s.rank * loc.shape[0]:(s.rank + 1) * loc.shape[0]].copy_(loc)
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


def simulate(groups_l, groups_h, widths, PB, P, K, bw_gbs):
    """Timeline of one rank: groups_l/h[hop][g] = light / hub ms."""
    main_t, comm_t = 0.0, 0.0
    arrive = [0.0] * len(widths)
    for h in range(K):
        new_arrive = []
        hub_end = 0.0
        for g, w in enumerate(widths):
            start = max(main_t, arrive[g])
            l_end = start + groups_l[h][g]
            h_end = start + groups_h[h][g]
            main_t = l_end
            hub_end = max(hub_end, h_end)
            if h < K - 1:  # exchanged
                a_start = max(l_end, h_end, comm_t)
                a = (P - 1) / P * PB * w * 4 / (bw_gbs * 1e9) * 1e3
                comm_t = a_start + a
                new_arrive.append(comm_t)
        arrive = new_arrive
        if h == K - 1:
            main_t = max(main_t, hub_end)
    return main_t


def simulate_chunks(gl, gh, RC, Bc, Fp, P, bw_gbs):
    """Timeline with row-chunked exchange: chunk c's all-gather (P*Bc rows x
    Fp) starts when its light and hub kernels are done; the next hop starts
    when every chunk has arrived.  gl/gh[hop] = per-launch ms (RC launches on
    exchanged hops, one on the last)."""
    t = 0.0
    for h in range(len(gl)):
        if h == len(gl) - 1:
            return t + max(gl[h][0], gh[h][0])
        main, comm = t, t
        for c in range(RC):
            end = main + gl[h][c]
            ready = max(end, t + gh[h][c])
            main = end
            comm = max(comm, ready) + (P - 1) / P * P * Bc * Fp * 4 / (bw_gbs * 1e9) * 1e3
        t = max(main, comm)
    return t


def parse_launches(light, hub, K, G):
    """Per-group light / hub ms from sgc_timing records: a split launch makes
    one record for the light kernel (hub None) and, when the rank has hub
    rows, one for the hub-only launch (its hub time set)."""
    gl = [[0.0] * G for _ in range(K)]
    gh = [[0.0] * G for _ in range(K)]
    i = 0
    for h in range(K):
        for g in range(G):
            if i < len(light) and hub[i] is None:
                gl[h][g] = light[i]
                i += 1
            if i < len(light) and hub[i] is not None:
                gh[h][g] = hub[i]
                i += 1
    return gl, gh


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="reddit")
    ap.add_argument("--layouts", default="2x1,4x1,8x1,2x2,4x2,2x4",
                    help="R x C: R row blocks x C feature blocks (P = R*C)")
    ap.add_argument("--group-floats", type=int, default=128)
    ap.add_argument("--bw", default="300,450,600", help="assumed all-gather ingress GB/s per rank")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--row-chunks", type=int, default=1,
                    help="exchanged hops in this many full-width row chunks (group floats 0)")
    ap.add_argument("--no-split", action="store_true",
                    help="hub rows inside each group launch (side stream, joined per launch)")
    args = ap.parse_args()
    spec = graphs.SHAPES[args.shape]
    S = graphs.synthetic_graph(args.shape, seed=0)
    F, K, n = spec["features"], spec["hops"], S.n
    X0 = torch.from_numpy(graphs.synthetic_features(args.shape, n, F, seed=1)).cuda()
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device="cuda")
    out = torch.empty((n, F), device="cuda")
    t1 = timeit(lambda: propagate(csr, X0, K, out=out), args.reps)
    print(json.dumps({"case": "single", "shape": args.shape, "ms": t1 * 1e3}), flush=True)
    rp = np.asarray(S.row_ptr, dtype=np.int64)
    bws = [float(b) for b in args.bw.split(",")]
    for lay in args.layouts.split(","):
        R, C = (int(x) for x in lay.split("x"))
        P = R * C
        for name, b in (("rows", equal_row_bounds(n, R)), ("nnz", nnz_balanced_bounds(rp, R))):
            loads = np.diff(rp[b])
            print(json.dumps({"case": "balance", "layout": lay, "bounds": name,
                              "max_over_mean_nnz": float(loads.max() / loads.mean()),
                              "max_over_mean_rows": float(np.diff(b).max() / np.diff(b).mean())}),
                  flush=True)
        fb, Bf = feature_bounds(F, C)
        ranks = []
        for i in range(R):
            shard = make_shard(S.row_ptr, S.col_idx, S.val, i, R, "cuda")
            for j in range(C):
                c0, c1 = int(fb[j]), int(fb[j + 1])
                Xj = X0[:, c0:c1]
                prop = LocalRowPropagator(shard, group_floats=args.group_floats,
                                          split_hubs=not args.no_split,
                                          row_chunks=args.row_chunks)
                t = timeit(lambda: prop.propagate(Xj, K, output="sharded"), args.reps)
                h0 = time.perf_counter()
                for _ in range(3):
                    prop.propagate(Xj, K, output="sharded")
                host = (time.perf_counter() - h0) / 3  # enqueue time (GPU still busy)
                torch.cuda.synchronize()
                collect_kernel_timing()
                kernel_timing(True)
                prop.propagate(Xj, K, output="sharded")
                kernel_timing(False)
                light, hub = collect_kernel_timing()
                Fw = (c1 - c0 + 31) // 32 * 32
                asm_bytes = (C - 1) * shard.rows * Bf * 4  # final tile assembly (C > 1)
                proj = {}
                # projected step = the rank's MEASURED compute-only wall time +
                # the exchange time the timeline model leaves exposed (model at
                # the given bandwidth minus the same model with a free exchange):
                # the kernel-time model alone ignores launch gaps and overlap
                # losses and reads optimistic for narrow groups
                if args.row_chunks > 1:
                    RC = args.row_chunks
                    Bc = -(-shard.block // RC)
                    gl = [[0.0] * RC for _ in range(K)]
                    gh = [[0.0] * RC for _ in range(K)]
                    recs = list(zip(light, hub))
                    i = 0
                    for h in range(K):
                        for c in range(RC if h < K - 1 else 1):
                            if i < len(recs) and recs[i][1] is None:
                                gl[h][c] = recs[i][0]
                                i += 1
                            if i < len(recs) and recs[i][1] is not None:
                                gh[h][c] = recs[i][1]
                                i += 1
                    free = simulate_chunks(gl, gh, RC, Bc, Fw, R, 1e9)
                    for bw in bws:
                        proj[f"{bw:g}GBps"] = (t * 1e3 + simulate_chunks(gl, gh, RC, Bc, Fw, R, bw)
                                               - free + asm_bytes / (bw * 1e9) * 1e3)
                else:
                    gfw = prop.group_floats or Fw
                    G = -(-Fw // gfw)
                    widths = [min(gfw, Fw - g * gfw) for g in range(G)]
                    gl, gh = parse_launches(light, hub, K, G)
                    free = simulate(gl, gh, widths, shard.gathered_rows, R, K, 1e9)
                    for bw in bws:
                        proj[f"{bw:g}GBps"] = (t * 1e3 + simulate(gl, gh, widths,
                                                                  shard.gathered_rows, R, K, bw)
                                               - free + asm_bytes / (bw * 1e9) * 1e3)
                rec = {"case": "rank", "layout": lay, "row_block": i, "col_block": j,
                       "rows": shard.rows, "nnz": shard.nnz, "cols": c1 - c0,
                       "compute_ms": t * 1e3, "host_enqueue_ms": host * 1e3,
                       "group_light_ms": gl, "group_hub_ms": gh, "proj_ms": proj}
                ranks.append(rec)
                print(json.dumps(rec), flush=True)
                del prop
            del shard
            torch.cuda.empty_cache()
        worst = max(r["compute_ms"] for r in ranks)
        proj = {k: max(r["proj_ms"][k] for r in ranks) for k in ranks[0]["proj_ms"]}
        ex = (R - 1) / R * n * ((F + 31) // 32 * 32 / C) * 4 * (K - 1)
        print(json.dumps({"case": "summary", "layout": lay, "P": P, "single_ms": t1 * 1e3,
                          "max_rank_compute_ms": worst,
                          "compute_only_speedup": t1 * 1e3 / worst,
                          "exchange_MB_per_rank": round(ex / 1e6, 1),
                          "projected_step_ms": proj,
                          "projected_speedup": {k: t1 * 1e3 / v for k, v in proj.items()},
                          "assumption": "all-gathers at the given per-rank ingress GB/s on one "
                                        "comm stream, overlapped as RowPartitionedPropagator "
                                        "does; kernel times measured on one GPU per rank"}),
              flush=True)


if __name__ == "__main__":
    main()
