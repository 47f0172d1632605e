"""RMAT-shape K=3 through the CPU twin (sgc_propagate_f32_cpu) against the
reference-generated golden hash (tests/golden/shapes.json "rmat").  Too large
for the CPU test suite (~3 minutes, ~30 GB); run by hand:

    python scripts/rmat_cpu_check.py      # log: profiles/r02_rmat_cpu_twin_check.log
"""
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from sgc_amd import graphs  # noqa: E402
from sgc_amd.propagate import DeviceCSR, propagate  # noqa: E402


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    g = json.load(open(os.path.join(ROOT, "tests/golden/shapes.json")))["rmat"]
    rows = dict(np.load(os.path.join(ROOT, "tests/golden/shape_rows.npz")))
    t = time.time()
    S = graphs.synthetic_graph("rmat", seed=g["seed"])
    print("graph", time.time() - t, flush=True)
    r, c, v = S.coo()
    print("indices", sha(np.stack([r, c])) == g["sha_indices"], "values",
          sha(v) == g["sha_values"], flush=True)
    del r, c, v
    X = graphs.synthetic_features("rmat", g["n"], g["features"], seed=g["feature_seed"])
    print("X", sha(X) == g["sha_X"], flush=True)
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device="cpu")
    t = time.time()
    Y = propagate(csr, torch.from_numpy(X), 3).numpy()
    dt = time.time() - t
    print("cpu twin K=3 %.1f s, %.3g edges/s (%d threads)" % (dt, 3 * S.nnz / dt,
                                                            torch.get_num_threads()), flush=True)
    print("rows", np.array_equal(Y[rows["rmat_rows"]].view(np.uint32),
                                 rows["rmat_K3"].view(np.uint32)))
    print("sha", sha(Y) == g["outputs"]["3"]["sha"])


if __name__ == "__main__":
    main()
