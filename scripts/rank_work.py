"""Per-rank compute of the N>1 paths, timed on ONE GPU (no exchange).

    python scripts/rank_work.py            # the per-rank step of each partition
    python scripts/rank_work.py --sweep    # one hop per case x schedule knobs

For P in {2, 4, 8}: what rank 0 (and the last rank) computes per step under
each partition of sgc_amd.distributed, at Reddit shape, K=2:
  features  column-block copy + K-1 full hops on the block + last hop in row
            chunks + the unpack of P gathered blocks into [N, F]
  rows      K hops over the rank's row block at full F (equal-row blocks)
The exchange itself (RCCL over xGMI) needs the 8-GPU node; this prices the
compute side of each design.  --sweep times ONE hop of: the full graph at
F=602, a 152- and a 76-column block over all rows, and a 1/8 row block at
F=602, for each (heavy, hub) threshold pair.  One JSON line per case.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sgc_amd import graphs  # noqa: E402
from sgc_amd.distributed import _copy_cols, equal_row_bounds, feature_bounds, row_chunks  # noqa: E402
from sgc_amd.propagate import DeviceCSR, aligned_ld, spmm  # noqa: E402


def timeit(fn, reps, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def sweep(csr, X0, n, F, reps, heavies, hubs):
    ld = aligned_ld(F)
    full = torch.empty((n, ld), device="cuda")
    _copy_cols(X0, full[:, :F])
    cases = [("full_F602", full[:, :F], 0, n)]
    for P in (4, 8):
        bounds, B = feature_bounds(F, P)
        blk = torch.empty((n, (B + 31) // 32 * 32), device="cuda")
        _copy_cols(X0[:, :int(bounds[1])], blk[:, :int(bounds[1])])
        cases.append((f"cols{int(bounds[1])}", blk[:, :int(bounds[1])], 0, n))
    rb = equal_row_bounds(n, 8)
    cases.append(("rows1of8_F602", full[:, :F], int(rb[0]), int(rb[1])))
    for name, X, r0, r1 in cases:
        out = torch.empty((r1 - r0, X.shape[1]), device="cuda")
        for th in heavies:
            for hb in hubs:
                pl = csr.plan(r0, r1, th, hb, X.shape[1])
                t = timeit(lambda: spmm(csr, X, r0, r1, out=out, threshold=th, hub_threshold=hb),
                           reps)
                nz = int((csr.row_ptr[r1] - csr.row_ptr[r0]).item())
                w = X.shape[1]
                gb = (4 * (r1 - r0 + 1) + 8 * nz + 4 * w * nz + 4 * w * (r1 - r0)) / 1e9
                print(json.dumps({"case": name, "heavy": th, "hub": hb, "n_heavy": pl.n_heavy,
                                  "n_hub": pl.n_hub, "hop_ms": t * 1e3,
                                  "gather_model_TBps": gb / t / 1e3}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="reddit")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--chunks", type=int, default=4)
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--heavy", default="auto")
    ap.add_argument("--hub", default="auto")
    args = ap.parse_args()
    spec = graphs.SHAPES[args.shape]
    S = graphs.synthetic_graph(args.shape, seed=0)
    F, K, n = spec["features"], spec["hops"], S.n
    X0 = torch.from_numpy(graphs.synthetic_features(args.shape, n, F, seed=1)).cuda()
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device="cuda")
    heavies = [None if x == "auto" else int(x) for x in args.heavy.split(",")]
    hubs = [None if x == "auto" else int(x) for x in args.hub.split(",")]
    if args.sweep:
        sweep(csr, X0, n, F, args.reps, heavies, hubs)
        return
    th, hb = heavies[0], hubs[0]
    ld = aligned_ld(F)
    full_a = torch.empty((n, ld), device="cuda")
    full_b = torch.empty((n, ld), device="cuda")
    out = torch.empty((n, F), device="cuda")

    def sp(X, r0, r1, o):
        return spmm(csr, X, r0, r1, out=o, threshold=th, hub_threshold=hb)

    def single():
        _copy_cols(X0, full_a[:, :F])
        sp(full_a[:, :F], 0, n, full_b[:, :F])
        sp(full_b[:, :F], 0, n, out)
    t1 = timeit(single, args.reps)
    print(json.dumps({"case": "single", "ms": t1 * 1e3}), flush=True)

    for P in (2, 4, 8):
        bounds, B = feature_bounds(F, P)
        for p in sorted({0, P - 1}):
            c0, c1 = int(bounds[p]), int(bounds[p + 1])
            w = c1 - c0
            ldb = (B + 31) // 32 * 32
            a = torch.empty((n, ldb), device="cuda")
            h = torch.empty((n, ldb), device="cuda")
            chunks = row_chunks(n, args.chunks)
            locs = [torch.empty((r1 - r0, B), device="cuda") for r0, r1 in chunks]
            fulls = [torch.empty((P * (r1 - r0), B), device="cuda") for r0, r1 in chunks]

            def hops():
                _copy_cols(X0[:, c0:c1], a[:, :w])
                src = a[:, :w]
                for _ in range(K - 1):
                    sp(src, 0, n, h[:, :w])
                    src = h[:, :w]
                for (r0, r1), loc in zip(chunks, locs):
                    sp(src, r0, r1, loc[:, :w])

            def unpack():
                for (r0, r1), fl in zip(chunks, fulls):
                    rows = r1 - r0
                    for q in range(P):
                        q0, q1 = int(bounds[q]), int(bounds[q + 1])
                        if q1 > q0:
                            _copy_cols(fl[q * rows:(q + 1) * rows, :q1 - q0], out[r0:r1, q0:q1])
            th_, tu = timeit(hops, args.reps), timeit(unpack, args.reps)
            print(json.dumps({"case": "features", "P": P, "rank": p, "cols": w,
                              "hops_ms": th_ * 1e3, "unpack_ms": tu * 1e3,
                              "speedup_vs_single_compute": t1 / (th_ + tu)}), flush=True)
        rb = equal_row_bounds(n, P)
        for p in sorted({0, P - 1}):
            r0, r1 = int(rb[p]), int(rb[p + 1])
            loc = torch.empty((r1 - r0, ld), device="cuda")

            def rows_hops():
                src = full_a[:, :F]
                for _ in range(K):
                    sp(src, r0, r1, loc[:, :F])
            tr = timeit(rows_hops, args.reps)
            print(json.dumps({"case": "rows", "P": P, "rank": p, "rows": r1 - r0,
                              "hops_ms": tr * 1e3, "speedup_vs_single_compute": t1 / tr}),
                  flush=True)


if __name__ == "__main__":
    main()
