"""Interleaved A/B of two builds of the library on one hop (or the K-hop loop).

    python scripts/lib_ab.py --libs A.so,B.so [--shape reddit] [--widths 76,128,F]
                             [--rounds 10] [--hops 1]

The first library also builds the CSR, the column groups and the plans; each
library then launches the same hops on the same inputs through its own
sgc_spmm_csr_f32_ex (round-robin, events on the launch stream, the hub
kernel's fork/join included), and every output is checked bit-identical to
the first library's.  Width W < F = one launch over all rows at W floats in
the engine's own 128-B-row buffers (the feature partition's per-rank hop);
F = the full width with the product's column-group rule.
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
from sgc_amd.propagate import (SPMM_ACCUMULATE, SPMM_X_PADDED, SPMM_Y_PADDED,  # noqa: E402
                               DeviceCSR, aligned_ld, column_groups_for, x_flags)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--shape", default="reddit")
    ap.add_argument("--widths", default="76,128,F")
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--hops", type=int, default=1)
    ap.add_argument("--groups", type=int, default=None, help="force G column groups")
    ap.add_argument("--ld", type=int, default=None, help="row stride of the buffers (floats)")
    args = ap.parse_args()
    paths = [os.path.abspath(p) for p in args.libs.split(",")]
    os.environ["SGC_AMD_LIB"] = paths[0]
    _lib.LIB_PATH = paths[0]
    libs = [_lib.load()] + [_lib.load_path(p) for p in paths[1:]]
    dev = torch.device("cuda", 0)
    S = graphs.synthetic_graph(args.shape, seed=0)
    F = graphs.SHAPES[args.shape]["features"]
    X0 = torch.from_numpy(graphs.synthetic_features(args.shape, S.n, F, seed=1)).to(dev)
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device=dev)
    stream = _lib.stream_handle(dev)
    for wtok in args.widths.split(","):
        w = F if wtok == "F" else int(wtok)
        ld = args.ld or aligned_ld(w)
        G = args.groups or column_groups_for(csr, w)
        parts = csr.column_groups(G) if G > 1 else [csr]
        plans = [c.plan(0, S.n, None, None, w) for c in parts]
        src = torch.zeros((S.n, ld), device=dev)
        src[:, :w] = X0[:, :w] if w <= F else 0
        bufs = [[torch.empty((S.n, ld), device=dev) for _ in range(2)] for _ in libs]

        def run(i):
            lib = libs[i]
            x = src
            for h in range(args.hops):
                y = bufs[i][h & 1]
                for g, (c, pl) in enumerate(zip(parts, plans)):
                    fl = (SPMM_X_PADDED | SPMM_Y_PADDED | x_flags(x[:, :w]) | pl.hub_flags() |
                          (SPMM_ACCUMULATE if g else 0))
                    rc = lib.sgc_spmm_csr_f32_ex(
                        _lib.ptr(c.row_ptr), _lib.ptr(c.col_idx), _lib.ptr(c.val), 0, S.n,
                        _lib.ptr(x), ld, _lib.ptr(y), ld, w, _lib.ptr(pl.rows), pl.n_heavy,
                        pl.n_hub, pl.threshold, fl, stream)
                    if rc:
                        raise RuntimeError(lib.sgc_last_error().decode())
                x = y
            return x

        outs = [run(i) for i in range(len(libs))]
        torch.cuda.synchronize()
        ref = outs[0][:, :w].cpu().numpy().view(np.uint32)
        same = [bool(np.array_equal(o[:, :w].cpu().numpy().view(np.uint32), ref)) for o in outs]
        times = [[] for _ in libs]
        for _ in range(args.rounds):
            for i in range(len(libs)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                run(i)
                e1.record()
                torch.cuda.synchronize()
                times[i].append(e0.elapsed_time(e1))
        rec = {"width": w, "groups": G, "hops": args.hops, "bit_identical": same,
               "ms_median": [round(float(np.median(t)), 4) for t in times],
               "ms_min": [round(float(np.min(t)), 4) for t in times],
               "libs": [os.path.relpath(p, ROOT) for p in paths]}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
