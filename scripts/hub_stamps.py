"""Where the hub chain's time goes: per-round clock stamps of block 0 of
spmm_hub_kernel (diagnostic build, -DSGC_HUB_STAMPS=1) on the largest row of
the Reddit-shape graph (47,857 nonzeros) alone, at HC = 64 and HC = 32.

    python -c "from sgc_amd import build; build.build(out='variants/stamps.so',
               defines=['SGC_HUB_STAMPS=1'])"
    SGC_AMD_LIB=variants/stamps.so python scripts/hub_stamps.py

Per round (a round = the nonzeros the 15 loader waves stage at once: 240 at
HC = 64, 480 at HC = 32), in shader cycles (s_memtime):
  chain   chain wave: barrier exit -> FMAs done (reaches the next barrier)
  wait    chain wave: FMAs done -> next barrier exit (waiting for loaders)
  store   loader wave 1: barrier exit -> its LDS store of the next round done
  issue   loader wave 1: store done -> reaches the barrier (X loads issued)
"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sgc_amd import _lib, graphs  # noqa: E402
from sgc_amd.propagate import DeviceCSR, spmm  # noqa: E402

ROUNDS = 4096


def main():
    S = graphs.synthetic_graph("reddit", seed=0)
    d = np.diff(S.row_ptr.astype(np.int64))
    r = int(np.argmax(d))
    nnz = int(d[r])
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device="cuda")
    lib = _lib.load()
    fn = lib.sgc_debug_hub_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    for hc, w in ((64, 64), (32, 32), (64, 602)):
        ld = (w + 31) // 32 * 32
        X = torch.randn((S.n, ld), device="cuda")
        Y = torch.empty((1, ld), device="cuda")
        lib.sgc_set_tuning(b"hub_chunk", hc)
        f = lambda: spmm(csr, X[:, :w], r, r + 1, out=Y[:, :w], threshold=1, hub_threshold=1)
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) * 1e6
        buf = (ctypes.c_ulonglong * (5 * ROUNDS))()
        _lib.check(fn(ctypes.cast(buf, ctypes.c_void_p), 5 * ROUNDS), "debug_hub_stamps")
        st = np.frombuffer(buf, dtype=np.uint64).reshape(5, ROUNDS).astype(np.int64)
        per_round = 240 if hc == 64 else 480
        nr = (nnz + per_round - 1) // per_round
        s0, s1, s2, s3 = (st[i, :nr] for i in range(4))
        chain = s1 - s0
        wait = s0[1:] - s1[:-1]
        store = s2[:-1] - s0[:-1]
        issue = s3 - s2
        clk = (st[4, 2] - st[4, 0]) / max(1, st[4, 3] - st[4, 1]) * 100e6
        kern_cycles = st[4, 2] - st[4, 0]
        rec = {"hc": hc, "width": w, "row_nnz": nnz, "rounds": nr, "host_us": round(us, 1),
               "kernel_cycles": int(kern_cycles), "clock_GHz": round(clk / 1e9, 3),
               "kernel_us_from_stamps": round(kern_cycles / clk * 1e6, 1),
               "chain_cycles_per_round_median": float(np.median(chain)),
               "wait_cycles_per_round_median": float(np.median(wait)),
               "loader_store_cycles_median": float(np.median(store)),
               "loader_issue_cycles_median": float(np.median(issue)),
               "chain_cycles_per_nonzero": float(np.median(chain)) / per_round,
               "round_cycles_per_nonzero": float(np.median(np.diff(s0))) / per_round,
               "chain_share": float(chain.sum()) / float(max(1, s0[-1] - s0[0] + chain[-1]))}
        print(json.dumps(rec), flush=True)
    lib.sgc_set_tuning(b"hub_chunk", 0)


if __name__ == "__main__":
    main()
