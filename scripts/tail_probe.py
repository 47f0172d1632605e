"""Is a narrow pass bounded by its longest rows?  (timing only)

    python scripts/tail_probe.py [--widths 64,76,32] [--cap 1000]

One hop over the Reddit-shape S at width W (engine buffers, one launch, the
product's plan) against the same hop over S' = S with every row longer than
`cap` cut into rows of at most `cap` nonzeros: the same nonzeros in the same
order, gathering the same X rows, but no FMA chain longer than `cap` (S'
computes different sums -- it is a probe of the schedule, not a result).
Also the pass split into feature blocks (e.g. 64 + 12) in separate packed
buffers, each block one launch.
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
from sgc_amd.propagate import SPMM_X_PADDED, SPMM_Y_PADDED, DeviceCSR, aligned_ld, spmm  # noqa: E402


def split_rows(row_ptr, cap):
    d = np.diff(row_ptr)
    pieces = np.maximum(1, (d + cap - 1) // cap)
    starts = []
    for r in np.flatnonzero(pieces > 1):
        starts.append((r, np.arange(row_ptr[r], row_ptr[r + 1], cap)))
    rp = list(row_ptr[:-1])
    extra = np.concatenate([s[1:] for _, s in starts]) if starts else np.array([], np.int64)
    rp = np.sort(np.concatenate([np.asarray(rp, np.int64), extra]))
    return np.concatenate([rp, [row_ptr[-1]]]).astype(np.int32)


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    ms = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ms.append(s.elapsed_time(e))
    return round(float(np.median(ms)), 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--widths", default="64,76,32,12")
    ap.add_argument("--splits", default="76=64+12,76=32+32+12,64=32+32")
    ap.add_argument("--cap", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    S = graphs.synthetic_graph("reddit", seed=0)
    X = torch.from_numpy(graphs.synthetic_features("reddit", S.n, 602, seed=1)).to(dev)
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device=dev)
    rp2 = split_rows(np.asarray(S.row_ptr, np.int64), a.cap)
    n2 = rp2.size - 1
    csr2 = DeviceCSR(n2, S.n, torch.from_numpy(rp2).to(dev), csr.col_idx, csr.val, csr.status)
    pad = SPMM_X_PADDED | SPMM_Y_PADDED
    bufs = {}

    def block(w):
        if w not in bufs:
            ld = aligned_ld(w)
            Xw = torch.zeros((S.n, ld), device=dev)
            Xw[:, :w] = X[:, :w]
            bufs[w] = (Xw, torch.empty((max(S.n, n2), ld), device=dev))
        return bufs[w]
    for w in (int(t) for t in a.widths.split(",")):
        Xw, Y = block(w)
        rec = {"width": w,
               "S_ms": timed(lambda: spmm(csr, Xw[:, :w], out=Y[:S.n, :w], flags=pad), a.reps),
               "S_split_rows_ms": timed(lambda: spmm(csr2, Xw[:, :w], out=Y[:n2, :w], flags=pad),
                                        a.reps),
               "cap": a.cap, "rows": S.n, "rows_split": n2}
        print(json.dumps(rec), flush=True)
    for spec in a.splits.split(","):
        w, parts = spec.split("=")
        parts = [int(p) for p in parts.split("+")]

        def run(c):
            for p in parts:
                Xp, Yp = block(p)
                spmm(c, Xp[:, :p], out=Yp[:c.n_rows, :p], flags=pad)
        print(json.dumps({"split": spec, "S_ms": timed(lambda: run(csr), a.reps),
                          "S_split_rows_ms": timed(lambda: run(csr2), a.reps)}), flush=True)


if __name__ == "__main__":
    main()
