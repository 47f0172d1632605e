"""A/B of the light-row order (SPMM_LIGHT_ORDER): the same launches with the
plan's light rows in length order vs row order, interleaved rounds, outputs
checked bit-identical.  Cases: the Reddit-shape K=2 propagate (N=1), one hop
of a 76-column block over all rows (a P=8 feature-partition rank), one hop
of a 1/8 row block at F=602 (a P=8 row-partition rank).  One JSON line each.
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import sgc_amd.propagate  # noqa: E402,F401
from sgc_amd import graphs  # noqa: E402
from sgc_amd.distributed import equal_row_bounds  # noqa: E402

pg = sys.modules["sgc_amd.propagate"]  # the module (the package exports a function of that name)


def main():
    S = graphs.synthetic_graph("reddit", seed=0)
    F = 602
    X = torch.from_numpy(graphs.synthetic_features("reddit", S.n, F, seed=1)).cuda()
    X76 = torch.zeros((S.n, 96), device="cuda")
    X76[:, :76] = X[:, :76]
    r1 = int(equal_row_bounds(S.n, 8)[1])
    csrs = {}
    for order in (False, True):
        pg.LIGHT_ORDER = order
        c = pg.DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device="cuda")
        c.plan(0, S.n, None, None, F)
        c.plan(0, S.n, None, None, 76)
        c.plan(0, r1, None, None, F)
        csrs[order] = c
    outs = {}
    cases = {
        "reddit_K2": lambda c, o: pg.propagate(c, X, 2, out=o),
        "w76_all_rows": lambda c, o: pg.spmm(c, X76[:, :76], 0, S.n, out=o[:, :76],
                                             flags=pg.SPMM_X_PADDED | pg.SPMM_Y_PADDED),
        "w602_rows_1of8": lambda c, o: pg.spmm(c, X, 0, r1, out=o[:r1]),
    }
    times = {(k, o): [] for k in cases for o in (False, True)}
    for k in cases:
        for o in (False, True):
            out = torch.empty((S.n, F), device="cuda")
            cases[k](csrs[o], out)
            torch.cuda.synchronize()
            outs[(k, o)] = out
        a, b = outs[(k, False)], outs[(k, True)]
        cols = 76 if k == "w76_all_rows" else F
        rows = r1 if k == "w602_rows_1of8" else S.n
        assert torch.equal(a[:rows, :cols], b[:rows, :cols]), k
    for _ in range(7):
        for k in cases:
            for o in (False, True):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(3):
                    cases[k](csrs[o], outs[(k, o)])
                e.record()
                e.synchronize()
                times[(k, o)].append(s.elapsed_time(e) / 3)
    for k in cases:
        t0, t1 = float(np.median(times[(k, False)])), float(np.median(times[(k, True)]))
        print(json.dumps({"case": k, "row_order_ms": round(t0, 4), "light_order_ms": round(t1, 4),
                          "speedup": round(t0 / t1, 4), "bit_identical": True}), flush=True)


if __name__ == "__main__":
    main()
