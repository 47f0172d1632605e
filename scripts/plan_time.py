import sys, time, os
sys.path.insert(0, os.getcwd())
import torch
import sgc_amd.propagate
pg = sys.modules["sgc_amd.propagate"]
from sgc_amd import graphs
S = graphs.synthetic_graph("reddit", seed=0)
torch.zeros(1, device="cuda"); torch.cuda.synchronize()
for order in (False, True, False, True):
    pg.LIGHT_ORDER = order
    c = pg.DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device="cuda")
    torch.cuda.synchronize()
    t = time.perf_counter(); c.plan(0, S.n, None, None, 602); torch.cuda.synchronize()
    print("order", order, "plan ms", round((time.perf_counter() - t) * 1e3, 2), flush=True)
