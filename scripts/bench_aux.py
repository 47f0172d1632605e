"""Timing of the §8(f) rows next to the hot path, Reddit shape, one GPU:

  normalize  host scipy AugNorm (the reference's normalization.py:5-12 +
             utils.py:23-30) vs the on-device path (sgc_augnorm_count/fill +
             COO export), both producing identical S
  train      one SGC closure at Reddit-train shape (152,410 x 602 -> 41):
             torch (nn.Linear + F.cross_entropy + backward), the MFMA forward
             + torch backward (sgc_amd.models.SGC), and the fused step
             (sgc_cross_entropy); then reddit.py's LBFGS (2 steps) both ways
Prints one JSON line per measurement.
"""
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from sgc_amd import graphs  # noqa: E402
from sgc_amd.models import SGC, sgc_cross_entropy  # noqa: E402
from sgc_amd.normalization import aug_normalize_on_device, aug_normalized_adjacency  # noqa: E402
from sgc_amd.propagate import to_torch_coo  # noqa: E402
from sgc_amd.utils import sparse_mx_to_torch_sparse_tensor  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    return float(np.median(ts))


def bench_normalize():
    spec = graphs.SHAPES["reddit"]
    u, v = graphs.rmat_pairs(spec["n"], spec["edges"], seed=0)
    A = sp.coo_matrix((np.ones(len(u)), (u, v)), shape=(spec["n"],) * 2).tocsr()
    A = A + A.T
    t = time.perf_counter()
    ref = sparse_mx_to_torch_sparse_tensor(aug_normalized_adjacency(A)).float().cuda()
    torch.cuda.synchronize()
    t_host = time.perf_counter() - t
    dev = timed(lambda: to_torch_coo(aug_normalize_on_device(A)), reps=3)
    got = to_torch_coo(aug_normalize_on_device(A))
    same = torch.equal(got._indices(), ref._indices()) and torch.equal(got._values(), ref._values())
    print(json.dumps({"what": "augnorm reddit-shape", "nnz": int(ref._nnz()),
                      "host_scipy_s": round(t_host, 3), "device_s": round(dev, 4),
                      "speedup": round(t_host / dev, 1), "bit_identical": bool(same)}), flush=True)


def bench_train():
    torch.manual_seed(0)
    M, K, C = 152410, 602, 41
    X = torch.randn(M, K, device="cuda")
    y = torch.randint(0, C, (M,), device="cuda")
    lin = torch.nn.Linear(K, C).cuda()
    m = SGC(K, C).cuda()
    m.W.load_state_dict(lin.state_dict())

    def torch_closure():
        lin.zero_grad()
        torch.nn.functional.cross_entropy(lin(X), y).backward()

    def mfma_closure():
        m.zero_grad()
        torch.nn.functional.cross_entropy(m(X), y).backward()

    def fused_closure():
        m.zero_grad()
        sgc_cross_entropy(m, X, y).backward()
    res = {k: timed(f, reps=20) * 1e3 for k, f in
           (("torch_ms", torch_closure), ("mfma_fwd_torch_bwd_ms", mfma_closure),
            ("fused_ms", fused_closure))}
    x_bytes = M * K * 4
    res["fused_x_reads_GBps"] = 2 * x_bytes / (res["fused_ms"] * 1e-3) / 1e9
    print(json.dumps({"what": "SGC closure fwd+bwd, reddit-train shape", "M": M, "K": K, "C": C,
                      **{k: round(v, 4) for k, v in res.items()}}), flush=True)

    def lbfgs(fused):
        mm = SGC(K, C).cuda()
        mm.W.load_state_dict(lin.state_dict())
        opt = torch.optim.LBFGS(mm.parameters(), lr=1)

        def closure():
            opt.zero_grad()
            loss = sgc_cross_entropy(mm, X, y) if fused else \
                torch.nn.functional.cross_entropy(mm(X), y)
            loss.backward()
            return loss
        for _ in range(2):
            opt.step(closure)
        return mm
    t_unf = timed(lambda: lbfgs(False), reps=3)
    t_f = timed(lambda: lbfgs(True), reps=3)
    print(json.dumps({"what": "reddit.py LBFGS 2 steps", "unfused_s": round(t_unf, 4),
                      "fused_s": round(t_f, 4)}), flush=True)


if __name__ == "__main__":
    which = sys.argv[1:] or ["normalize", "train"]
    if "normalize" in which:
        bench_normalize()
    if "train" in which:
        bench_train()
