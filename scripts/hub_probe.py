"""Latency floor of one hub row: SpMM over ONLY the largest row of the
Reddit-shape graph (47,857 nonzeros), so the launch time is that row's
sequential FMA chain (+ launch overhead) -- per feature width, on the hub
kernel (HC 32 / 64) and as heavy items.  One JSON line per case.
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sgc_amd import _lib, graphs  # noqa: E402
from sgc_amd.propagate import DeviceCSR, spmm  # noqa: E402


def main():
    S = graphs.synthetic_graph("reddit", seed=0)
    d = np.diff(S.row_ptr.astype(np.int64))
    r = int(np.argmax(d))
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device="cuda")
    lib = _lib.load()
    widths = [int(x) for x in os.environ.get("HUB_PROBE_WIDTHS", "32,64,128,320,602").split(",")]
    modes = os.environ.get("HUB_PROBE_MODES", "hub64,hub32,heavy,light").split(",")
    lib_name = os.path.basename(_lib.LIB_PATH)
    for w in widths:
        ld = (w + 31) // 32 * 32
        X = torch.randn((S.n, ld), device="cuda")
        Y = torch.empty((1, ld), device="cuda")
        for mode, th, hb, hc in (("hub64", 1, 1, 64), ("hub32", 1, 1, 32), ("heavy", 1, 10**9, 0),
                                 ("light", 10**9, 10**9, 0)):
            if mode not in modes:
                continue
            lib.sgc_set_tuning(b"hub_chunk", hc)
            f = lambda: spmm(csr, X[:, :w], r, r + 1, out=Y[:, :w], threshold=th, hub_threshold=hb)
            for _ in range(3):
                f()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                f()
            torch.cuda.synchronize()
            us = (time.perf_counter() - t0) / 20 * 1e6
            print(json.dumps({"lib": lib_name, "row_nnz": int(d[r]), "width": w, "mode": mode,
                              "us": round(us, 1),
                              "ns_per_nonzero": round(us * 1e3 / d[r], 2)}), flush=True)
        lib.sgc_set_tuning(b"hub_chunk", 0)


if __name__ == "__main__":
    main()
