"""Where a narrow feature-block pass spends its time.

    python scripts/narrow_pass.py [--widths 76,128,152] [--reps 20] [--only W]

One SpMM launch over ALL rows of the Reddit-shape S at width W (the feature
partition's per-rank hop at P = 602 / W), in the engine's own 128-B-row
buffers (pad flags), timed by the library's own events: the light/heavy
kernel and the hub kernel on their streams, and the launch span.  Also the
light kernel with the hub rows cut out (SGC_SPMM_NO_HUB) and the hub rows
alone (SGC_SPMM_HUB_ONLY), so the tail each part leaves is visible.  --only W
loops one full launch (for rocprofv3 --pmc passes).
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from sgc_amd import graphs  # noqa: E402
from sgc_amd.propagate import (SPMM_HUB_ONLY, SPMM_NO_HUB, SPMM_X_PADDED,  # noqa: E402
                               SPMM_Y_PADDED, DeviceCSR, collect_launch_timing,
                               kernel_timing, spmm)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--widths", default="76,128,152")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", type=int, default=None)
    ap.add_argument("--loops", type=int, default=50)
    ap.add_argument("--heavy", type=int, default=None)
    ap.add_argument("--hub", type=int, default=None)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    S = graphs.synthetic_graph("reddit", seed=0)
    X = torch.from_numpy(graphs.synthetic_features("reddit", S.n, 602, seed=1)).to(dev)
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device=dev)
    widths = [args.only] if args.only else [int(w) for w in args.widths.split(",")]
    pad = SPMM_X_PADDED | SPMM_Y_PADDED
    for w in widths:
        ld = (w + 31) // 32 * 32
        Xw = torch.zeros((S.n, ld), device=dev)
        Xw[:, :w] = X[:, :w]
        Y = torch.empty((S.n, ld), device=dev)
        kw = dict(threshold=args.heavy, hub_threshold=args.hub)
        pl = csr.plan(0, S.n, args.heavy, args.hub, w)
        variants = {"full": pad, "light_only": pad | SPMM_NO_HUB, "hub_only": pad | SPMM_HUB_ONLY}
        for fl in variants.values():
            spmm(csr, Xw[:, :w], out=Y[:, :w], flags=fl, **kw)
        torch.cuda.synchronize()
        if args.only:
            for _ in range(args.loops):
                spmm(csr, Xw[:, :w], out=Y[:, :w], flags=pad, **kw)
            torch.cuda.synchronize()
            print(json.dumps({"width": w, "loops": args.loops}))
            return
        res = {k: {"light": [], "hub": [], "span": []} for k in variants}
        collect_launch_timing()
        kernel_timing(True)
        for _ in range(args.reps):
            for name, fl in variants.items():  # interleaved
                spmm(csr, Xw[:, :w], out=Y[:, :w], flags=fl, **kw)
                torch.cuda.synchronize()
                light, hub, span, kind = collect_launch_timing()
                res[name]["light"].append(light[-1])
                res[name]["hub"].append(hub[-1] if hub[-1] is not None else 0.0)
                res[name]["span"].append(span[-1])
        kernel_timing(False)
        rec = {"width": w, "ld": ld, "heavy_threshold": pl.threshold, "n_heavy": pl.n_heavy,
               "n_hub": pl.n_hub, "max_hub_degree": pl.max_hub_degree, "kernel": kind[-1]}
        for name in variants:
            rec[name] = {k: round(float(np.median(v)), 4) for k, v in res[name].items()}
        nnz = S.nnz
        rec["light_only_Gnnz_per_s"] = round(nnz / rec["light_only"]["light"] / 1e6, 2)
        rec["gather_TBps_full"] = round(4 * w * nnz / rec["full"]["span"] / 1e9, 2)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
