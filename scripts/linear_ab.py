"""Interleaved A/B of the classifier forward kernels at Reddit-train shape.

    python scripts/linear_ab.py [--rows 152410] [--features 602] [--classes 41]
                                [--kernels 2,5,6] [--rounds 5]

Each round times every `linear_kernel` tuning value (sgc_set_tuning: 1 LDS
tile, 2 fp32 streaming, 5 split-bf16 streaming, 6 its loads-only DIAG form)
with events over --reps forwards; prints the per-kernel median over rounds,
the HBM fraction of the algorithmic bytes (X once, Y once, W once) and the
largest error against fp64 for the non-DIAG forms.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sgc_amd import _lib  # noqa: E402
from sgc_amd.propagate import linear  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=152410)
    ap.add_argument("--features", type=int, default=602)
    ap.add_argument("--classes", type=int, default=41)
    ap.add_argument("--kernels", default="2,5,6")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    lib = _lib.load()
    M, K, C = a.rows, a.features, a.classes
    g = torch.Generator().manual_seed(0)
    x = torch.randn(M, K, generator=g).cuda()
    W = (torch.randn(C, K, generator=g) * 0.05).cuda()
    b = torch.randn(C, generator=g).cuda()
    ref = torch.nn.functional.linear(x.double(), W.double(), b.double())
    kernels = [int(k) for k in a.kernels.split(",")]
    times = {k: [] for k in kernels}
    errs = {}
    out = torch.empty((M, C), device="cuda")
    nbytes = 4 * M * K + 4 * M * C + 4 * C * K
    try:
        for _ in range(a.rounds):
            for k in kernels:
                _lib.check(lib.sgc_set_tuning(b"linear_kernel", k), "set_tuning")
                for _ in range(3):
                    linear(x, W, b, out=out)
                torch.cuda.synchronize()
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(a.reps)]
                for s, e in ev:
                    s.record()
                    linear(x, W, b, out=out)
                    e.record()
                torch.cuda.synchronize()
                times[k].append(float(np.median([s.elapsed_time(e) for s, e in ev])))
                if k not in (3, 4, 6, 7, 8) and k not in errs:
                    errs[k] = (out.double() - ref).abs().max().item()
    finally:
        lib.sgc_set_tuning(b"linear_kernel", 0)
    for k in kernels:
        _lib.check(lib.sgc_set_tuning(b"linear_kernel", k), "set_tuning")
        name = lib.sgc_linear_kernel_name(M, K, x.stride(0), C, _lib.ptr(x)).decode()
        lib.sgc_set_tuning(b"linear_kernel", 0)
        ms = float(np.median(times[k]))
        print(json.dumps({"linear_kernel": k, "kernel": name, "ms_median": ms,
                          "ms_rounds": [round(t, 4) for t in times[k]],
                          "TBps": nbytes / ms / 1e9, "frac": nbytes / ms / 1e9 / 8.0,
                          "max_abs_err_vs_fp64": errs.get(k)}), flush=True)


if __name__ == "__main__":
    main()
