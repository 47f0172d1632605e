"""Interleaved A/B of X_0's re-layout before hop 1.

    python scripts/pad_ab.py [--shape reddit] [--rounds 10] [--steps 5]

The public K-hop call at BASELINE shape, alternating per round between
propagate.PAD_X0 = True (pad_rows_kernel copies X_0 into 128-B rows, ld 608 at
Reddit, and hop 1 gathers with 16-B lanes) and False (hop 1 reads the
caller's ld-602 rows in place: 8-B lanes), `--steps` calls per round timed
with events; every output checked bit-identical to the first.  Prints the
per-mode medians and the per-round pairs.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import importlib  # noqa: E402

from sgc_amd import graphs  # noqa: E402

P = importlib.import_module("sgc_amd.propagate")  # the module (sgc_amd.propagate is also a function name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="reddit")
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    spec = graphs.SHAPES[a.shape]
    S = graphs.synthetic_graph(a.shape, seed=0)
    X = torch.from_numpy(graphs.synthetic_features(a.shape, S.n, spec["features"], seed=1)).cuda()
    csr = P.DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device="cuda")
    K = spec["hops"]
    ref = None
    times = {True: [], False: []}
    for r in range(a.rounds + 1):
        for mode in (True, False) if r % 2 == 0 else (False, True):
            P.PAD_X0 = mode
            out = P.propagate(csr, X, K)
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            assert torch.equal(out, ref), "re-layout changed the result"
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.steps):
                P.propagate(csr, X, K)
            e.record()
            torch.cuda.synchronize()
            if r:
                times[mode].append(s.elapsed_time(e) / a.steps)
    P.PAD_X0 = None
    print(json.dumps({"shape": a.shape, "K": K, "ld_x0": X.stride(0),
                      "pad_ms_median": float(np.median(times[True])),
                      "inplace_ms_median": float(np.median(times[False])),
                      "pad_ms": [round(t, 4) for t in times[True]],
                      "inplace_ms": [round(t, 4) for t in times[False]],
                      "bit_identical": True, "rule_pads": bool(P.pad_pays(csr, X.shape[1]))}),
          flush=True)


if __name__ == "__main__":
    main()
