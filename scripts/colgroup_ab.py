"""Column-group passes at N = 1: does a smaller live X raise the L2 hit rate
enough to pay for the extra passes?

    python scripts/colgroup_ab.py [--shape reddit] [--groups 1,2,4,8]

S is split into G groups of columns (equal nonzeros); one hop is then G
launches over all rows, group 0 plain and groups 1.. with
SGC_SPMM_ACCUMULATE, which continues every row's FMA chain from the value
the previous group's launch stored (CSR rows have ascending columns, so the
order of the chain is unchanged and the result is bit-identical).  Each
launch gathers only X rows of its group: at G = 8 the live part of a
128-float slice is 15 MB instead of 119 MB.  Interleaved rounds, one hop at
the full width in the engine's padded buffers; output checked bit-identical
to G = 1.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sgc_amd import graphs  # noqa: E402
from sgc_amd.propagate import (SPMM_ACCUMULATE, SPMM_X_PADDED, SPMM_Y_PADDED,  # noqa: E402
                               DeviceCSR, spmm)


def column_split(S, G):
    """G sub-CSRs over all rows, columns split at equal nonzero counts."""
    cnt = np.bincount(S.col_idx, minlength=S.n).astype(np.int64)
    cum = np.cumsum(cnt)
    cuts = [0] + [int(np.searchsorted(cum, S.nnz * g / G)) for g in range(1, G)] + [S.n]
    grp = np.searchsorted(np.asarray(cuts[1:]), S.col_idx, side="right")
    row = np.repeat(np.arange(S.n), np.diff(S.row_ptr))
    out = []
    for g in range(G):
        m = grp == g
        rp = np.zeros(S.n + 1, np.int64)
        np.cumsum(np.bincount(row[m], minlength=S.n), out=rp[1:])
        out.append(DeviceCSR.from_host_arrays(rp.astype(np.int32), S.col_idx[m], S.val[m],
                                              n_cols=S.n, device="cuda"))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="reddit")
    ap.add_argument("--groups", default="1,2,4,8")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--widths", default="F", help="comma list of launch widths (F = the shape's)")
    args = ap.parse_args()
    S = graphs.synthetic_graph(args.shape, seed=0)
    subs = {G: column_split(S, G) for G in (int(g) for g in args.groups.split(","))}
    for w in args.widths.split(","):
        F = graphs.SHAPES[args.shape]["features"] if w == "F" else int(w)
        one_width(args, S, F, subs)


def one_width(args, S, F, subs):
    ld = (F + 31) // 32 * 32
    X = torch.zeros((S.n, ld), device="cuda")
    X[:, :F] = torch.randn((S.n, F), generator=torch.Generator().manual_seed(1)).cuda()
    Y = torch.empty((S.n, ld), device="cuda")

    def run(G):
        for g, c in enumerate(subs[G]):
            spmm(c, X[:, :F], 0, S.n, out=Y[:, :F],
                 flags=SPMM_X_PADDED | SPMM_Y_PADDED | (SPMM_ACCUMULATE if g else 0))
    outs = {}
    for G in subs:
        run(G)
        torch.cuda.synchronize()
        outs[G] = Y[:, :F].clone()
    ms = {G: [] for G in subs}
    for _ in range(args.rounds):
        for G in subs:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            run(G)
            e.record()
            torch.cuda.synchronize()
            ms[G].append(s.elapsed_time(e))
    first = next(iter(subs))
    for G in subs:
        print(json.dumps({"shape": args.shape, "groups": G, "F": F,
                          "bit_identical": bool(torch.equal(outs[G], outs[first])),
                          "hop_median_ms": round(float(np.median(ms[G])), 4),
                          "hop_min_ms": round(float(np.min(ms[G])), 4)}), flush=True)


if __name__ == "__main__":
    main()
