"""Interleaved A/B of one schedule knob (sgc_set_tuning) on the product path.

    python scripts/ab_tune.py --knob heavy_pairs --values 0,1 [--shape reddit]
                              [--widths F,76] [--rounds 8]

For each width W (F = the shape's full width through sgc_precompute's engine,
propagate(); a narrower W = one SpMM launch over all rows at that width in
the engine's own padded buffers -- the feature partition's per-rank hop), the
knob's values are timed round-robin in one process (events on the launch
stream), and every value's output is checked bit-identical to the first's.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from sgc_amd import _lib, graphs  # noqa: E402
from sgc_amd.propagate import SPMM_X_PADDED, SPMM_Y_PADDED, DeviceCSR, propagate, spmm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--knob", default="heavy_pairs")
    ap.add_argument("--values", default="0,1")
    ap.add_argument("--shape", default="reddit")
    ap.add_argument("--widths", default="F,76")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--rows", default="all", help="all, or P:p = rank p's 1/P nnz-balanced rows")
    ap.add_argument("--attr", default=None,
                    help="A/B a module attribute of sgc_amd.propagate (e.g. COLUMN_GROUPS; "
                         "values as ints) instead of a knob")
    ap.add_argument("--kwarg", default=None,
                    help="A/B a keyword of spmm() (threshold, hub_threshold) instead of a knob; "
                         "-1 = the default")
    args = ap.parse_args()
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    S = graphs.synthetic_graph(args.shape, seed=0)
    F = graphs.SHAPES[args.shape]["features"]
    K = graphs.SHAPES[args.shape]["hops"]
    X = torch.from_numpy(graphs.synthetic_features(args.shape, S.n, F, seed=1)).to(dev)
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device=dev)
    values = [int(v) for v in args.values.split(",")]
    r0, r1 = 0, S.n
    if args.rows != "all":
        from sgc_amd.distributed import nnz_balanced_bounds
        P, p = (int(x) for x in args.rows.split(":"))
        b = nnz_balanced_bounds(S.row_ptr, P)
        r0, r1 = int(b[p]), int(b[p + 1])
    cur = {"v": -1}
    for wspec in args.widths.split(","):
        if wspec == "F" and args.rows == "all":
            out = torch.empty_like(X)

            def run():
                propagate(csr, X, K, out=out)
                return out
            label = f"{args.shape} propagate K={K} (F={F})"
        else:
            w = F if wspec == "F" else int(wspec)
            ld = (w + 31) // 32 * 32
            Xw = torch.zeros((S.n, ld), device=dev)
            Xw[:, :w] = X[:, :w]
            Y = torch.empty((r1 - r0, ld), device=dev)

            def run(Xw=Xw, Y=Y, w=w):
                kw = {}
                if args.kwarg and cur["v"] >= 0:
                    kw[args.kwarg] = cur["v"]
                spmm(csr, Xw[:, :w], r0, r1, out=Y[:, :w], flags=SPMM_X_PADDED | SPMM_Y_PADDED,
                     **kw)
                return Y[:, :w]
            label = f"one hop, width {w}, rows [{r0}, {r1})"
        ms = {v: [] for v in values}
        outs = {}

        def select(v):
            if args.attr:
                import importlib
                setattr(importlib.import_module("sgc_amd.propagate"), args.attr, v)
            elif args.kwarg:
                cur["v"] = v
            else:
                _lib.check(lib.sgc_set_tuning(args.knob.encode(), v), "set_tuning")
        for v in values:  # warm-up: plans, code objects
            select(v)
            outs[v] = run().clone()
        torch.cuda.synchronize()
        for _ in range(args.rounds):
            for v in values:
                select(v)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                run()
                e.record()
                torch.cuda.synchronize()
                ms[v].append(s.elapsed_time(e))
        same = all(torch.equal(outs[v], outs[values[0]]) for v in values)
        rec = {"case": label, "knob": args.attr or args.kwarg or args.knob,
               "bit_identical": bool(same)}
        for v in values:
            rec[f"{v}_median_ms"] = round(float(np.median(ms[v])), 4)
            rec[f"{v}_min_ms"] = round(float(np.min(ms[v])), 4)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
