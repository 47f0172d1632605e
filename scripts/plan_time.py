"""First-plan cost with and without the light order (SPMM_LIGHT_ORDER) in a
fresh process, after the library's code object is loaded (a tiny plan on
another graph first), as bench.py's first call meets it.  argv[1] = the
order of the first Reddit plan: "order" or "rows"."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sgc_amd.propagate  # noqa: E402,F401
from sgc_amd import graphs  # noqa: E402

pg = sys.modules["sgc_amd.propagate"]
first = sys.argv[1] if len(sys.argv) > 1 else "order"
S = graphs.synthetic_graph("reddit", seed=0)
T = graphs.synthetic_graph("cora", seed=0)
torch.zeros(1, device="cuda")
pg.LIGHT_ORDER = False
pg.DeviceCSR.from_host_arrays(T.row_ptr, T.col_idx, T.val, device="cuda").plan(0, T.n, None, None, 64)
torch.cuda.synchronize()
seq = (True, False, True, False) if first == "order" else (False, True, False, True)
for order in seq:
    pg.LIGHT_ORDER = order
    c = pg.DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device="cuda")
    torch.cuda.synchronize()
    t = time.perf_counter()
    c.plan(0, S.n, None, None, 602)
    torch.cuda.synchronize()
    print("order", order, "plan ms", round((time.perf_counter() - t) * 1e3, 2), flush=True)
