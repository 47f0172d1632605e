"""Timing of the SGC classifier at Reddit-train shape (reference models.py:7-18
and the training closure of reddit.py:51-64 / citation.py:35-58).

Used by bench.py (its `classifier` sub-record) and runnable on its own:

    python -m sgc_amd.classifier_bench [--rows 152410] [--features 602] [--classes 41]

Times, with events on the current stream, medians over --reps (forward and
backward: per call over 10 back-to-back calls, the kernels' own time; the
single-call figure, launch gap included, beside it):
  forward       SGC.forward on ROCm = sgc_linear_f32 (fp32 MFMA), and torch's
                F.linear beside it;
  backward      the weight gradients of the forward (sgc_linear_backward_f32:
                dW = dY^T X and db from one read of X) and torch's two ops;
  closure       the reference closure as written -- zero_grad,
                F.cross_entropy(model(x), y), backward -- with the drop-in SGC
                and with a plain nn.Linear (torch), and the fused
                sgc_cross_entropy step;
  lbfgs         reddit.py's train_regression: optim.LBFGS(lr=1), `epochs`
                steps of that closure (wall time, synchronised), drop-in SGC
                vs nn.Linear.
Bytes per launch: the forward reads X (M x F fp32) once and writes the logits;
the backward reads X and dY once.  frac = bytes / time / 8 TB/s.
"""
import argparse
import json
import time

import numpy as np
import torch
import torch.nn.functional as F
from torch import optim

HBM_PEAK_GBS = 8000.0


def _median_ms(fn, reps, warmup=3, inner=1):
    """Median over `reps` event pairs of the time per call, each pair around
    `inner` back-to-back calls (inner > 1: the launch gap between calls is
    hidden, so the figure is the kernels' own time, as rocprofv3 reports it)."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ms = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(inner):
            fn()
        e.record()
        torch.cuda.synchronize()
        ms.append(s.elapsed_time(e) / inner)
    return float(np.median(ms))


def _lbfgs_seconds(model, x, y, epochs):
    optimizer = optim.LBFGS(model.parameters(), lr=1)
    calls = [0]

    def closure():
        calls[0] += 1
        optimizer.zero_grad()
        loss = F.cross_entropy(model(x), y)
        loss.backward()
        return loss
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(epochs):
        optimizer.step(closure)
    torch.cuda.synchronize()
    return time.perf_counter() - t, calls[0]


def classifier_record(dev, M=152410, K=602, C=41, reps=20, epochs=2, seed=0):
    from .models import SGC, sgc_cross_entropy
    from .propagate import linear, linear_backward, warmup
    warmup(dev)
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(M, K, generator=g).to(dev)
    # learnable labels (a noisy linear teacher), so LBFGS runs its iterations
    # the way it does on reddit.py's data instead of stopping at once
    teacher = torch.randn(C, K, generator=g).to(dev) / K ** 0.5
    y = (x @ teacher.t() + 0.5 * torch.randn(M, C, generator=g).to(dev)).argmax(1)
    torch.manual_seed(seed)
    model = SGC(K, C).to(dev)
    ref = torch.nn.Linear(K, C).to(dev)
    with torch.no_grad():
        ref.weight.copy_(model.W.weight)
        ref.bias.copy_(model.W.bias)
    W, b = model.W.weight.detach(), model.W.bias.detach()
    dY = torch.randn(M, C, generator=g).to(dev)
    rec = {"shape": {"rows": M, "features": K, "classes": C},
           "what": "Reddit-train shape (reddit.py:45-49 train rows, models.py:7-18)"}
    fwd_bytes = 4 * M * K + 4 * M * C + 4 * C * K
    bwd_bytes = 4 * M * K + 4 * M * C
    t = _median_ms(lambda: linear(x, W, b), reps, inner=10)
    t1 = _median_ms(lambda: linear(x, W, b), reps)
    from . import _lib
    kname = _lib.load().sgc_linear_kernel_name(M, K, x.stride(0), C, _lib.ptr(x)).decode()
    rec["forward"] = {"kernel": f"{kname} (sgc_linear_f32; name from sgc_linear_kernel_name)",
                      "ms": t, "single_call_ms": t1,
                      "bytes": fwd_bytes, "achieved_GBps": fwd_bytes / t / 1e6,
                      "frac": fwd_bytes / t / 1e6 / HBM_PEAK_GBS,
                      "torch_F_linear_ms": _median_ms(lambda: F.linear(x, W, b), reps, inner=10)}
    t = _median_ms(lambda: linear_backward(x, dY), reps, inner=10)
    t1 = _median_ms(lambda: linear_backward(x, dY), reps)
    bname = _lib.load().sgc_linear_backward_kernel_name(M, K, x.stride(0), C, _lib.ptr(x)).decode()
    rec["backward"] = {"kernel": f"{bname} + reduction (sgc_linear_backward_f32; name from "
                                 "sgc_linear_backward_kernel_name)", "ms": t,
                       "single_call_ms": t1,
                       "bytes": bwd_bytes, "achieved_GBps": bwd_bytes / t / 1e6,
                       "frac": bwd_bytes / t / 1e6 / HBM_PEAK_GBS,
                       "torch_ms": _median_ms(lambda: (dY.t() @ x, dY.sum(0)), reps, inner=10)}

    def closure(m, fused=False):
        def run():
            m.zero_grad(set_to_none=False)
            loss = sgc_cross_entropy(m, x, y) if fused else F.cross_entropy(m(x), y)
            loss.backward()
            return loss
        return run
    rec["closure"] = {"dropin_ms": _median_ms(closure(model), reps),
                      "torch_nn_linear_ms": _median_ms(closure(ref), reps),
                      "fused_sgc_cross_entropy_ms": _median_ms(closure(model, fused=True), reps),
                      "what": "optimizer.zero_grad(); F.cross_entropy(model(x), y).backward() "
                              "(reddit.py:54-59), GPU time per call"}
    import copy
    init = copy.deepcopy(model.W.state_dict())
    for name, make in (("dropin", lambda: SGC(K, C).to(dev)),
                       ("torch_nn_linear", lambda: torch.nn.Linear(K, C).to(dev))):
        for rep in range(2):  # the first run warms the optimiser's code paths
            m = make()
            (m.W if hasattr(m, "W") else m).load_state_dict(init)
            s, calls = _lbfgs_seconds(m, x, y, epochs)
        rec.setdefault("lbfgs", {})[f"{name}_ms"] = s * 1e3
        rec["lbfgs"][f"{name}_closures"] = calls
    rec["lbfgs"]["what"] = (f"reddit.py train_regression: optim.LBFGS(lr=1), {epochs} steps, "
                            "wall time (synchronised)")
    return rec


def workload(dev, M=152410, K=602, C=41, loops=20):
    """Only the two classifier kernels, `loops` times each (rocprofv3 passes)."""
    from .propagate import linear, linear_backward
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(M, K, generator=g).to(dev)
    W = (torch.randn(C, K, generator=g) * 0.05).to(dev)
    b = torch.randn(C, generator=g).to(dev)
    dY = torch.randn(M, C, generator=g).to(dev)
    for _ in range(loops):
        linear(x, W, b)
        linear_backward(x, dY)
    torch.cuda.synchronize()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=152410)
    ap.add_argument("--features", type=int, default=602)
    ap.add_argument("--classes", type=int, default=41)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--workload", action="store_true", help="kernels only (profiling)")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="sgc_set_tuning before timing (e.g. tile_buffers=1)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    if a.tune:
        from . import _lib
        lib = _lib.load()
        for kv in a.tune:
            k, v = kv.split("=")
            _lib.check(lib.sgc_set_tuning(k.encode(), int(v)), "set_tuning")
    if a.workload:
        workload(dev, a.rows, a.features, a.classes)
        return
    print(json.dumps(classifier_record(dev, a.rows, a.features, a.classes, a.reps)), flush=True)


if __name__ == "__main__":
    main()
