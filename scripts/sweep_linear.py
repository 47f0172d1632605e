"""Interleaved timing of classifier-kernel build variants in one process
(Reddit-train shape 152,410 x 602 -> 41): sgc_linear_f32 and
sgc_linear_xent_f32.  Usage: python scripts/sweep_linear.py lib_a.so lib_b.so ..."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from sgc_amd import _lib  # noqa: E402


def main():
    libs = [_lib.LIB_PATH] + sys.argv[1:]
    loaded = [(os.path.basename(p), _lib.load_path(p)) for p in libs]
    M, K, C = 152410, 602, 41
    torch.manual_seed(0)
    X = torch.randn(M, K, device="cuda")
    W = torch.randn(C, K, device="cuda") * 0.05
    b = torch.randn(C, device="cuda")
    y = torch.randint(0, C, (M,), device="cuda")
    Y = torch.empty(M, C, device="cuda")
    loss = torch.empty((), device="cuda")
    dW = torch.empty_like(W)
    db = torch.empty_like(b)
    s = _lib.stream_handle()
    res = {}
    for name, lib in loaded:
        wsb = lib.sgc_linear_xent_workspace(M, K, C)
        ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
        res[name] = (lib, ws, wsb, {"linear": [], "xent": []})
    P = _lib.ptr
    for _ in range(8):
        for name, (lib, ws, wsb, t) in res.items():
            for what in ("linear", "xent"):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    if what == "linear":
                        rc = lib.sgc_linear_f32(P(X), K, P(W), P(b), P(Y), C, M, K, C, s)
                    else:
                        rc = lib.sgc_linear_xent_f32(P(X), K, P(W), P(b), P(y), M, K, C, P(loss),
                                                     P(dW), P(db), None, 0, P(ws), wsb, s)
                    assert rc == 0, lib.sgc_last_error()
                e1.record()
                e1.synchronize()
                t[what].append(e0.elapsed_time(e1) / 5)
    for name, (_, _, _, t) in res.items():
        print(json.dumps({"lib": name, **{k: round(float(np.median(v)) * 1e3, 1) for k, v in t.items()},
                          "unit": "us"}))


if __name__ == "__main__":
    main()
