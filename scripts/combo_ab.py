"""Interleaved A/B of schedule-knob COMBINATIONS on the K-hop propagation.

    python scripts/combo_ab.py --shape pubmed \\
        --configs "base:;r4:rows_per_wave=4;r4x:rows_per_wave=4,xcd_slices=1" [--rounds 10]

Each config is a name and sgc_set_tuning assignments (knobs the results never
depend on).  Per round every config runs --steps propagations of the shape's
K hops (propagate(), the engine under sgc_precompute), timed with events; every
output is checked bit-identical to the first config's.  One JSON line: the
per-config medians and rounds.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sgc_amd import _lib, graphs  # noqa: E402
from sgc_amd.propagate import DeviceCSR, propagate  # noqa: E402


def parse(spec):
    out = []
    for part in spec.split(";"):
        name, _, kv = part.partition(":")
        knobs = [(k, int(v)) for k, v in (x.split("=") for x in kv.split(",") if x)]
        out.append((name, knobs))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="pubmed")
    ap.add_argument("--configs", required=True)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    lib = _lib.load()
    configs = parse(a.configs)
    knobs = sorted({k for _, kv in configs for k, _ in kv})
    defaults = {k: lib.sgc_get_tuning(k.encode()) for k in knobs}
    spec = graphs.SHAPES[a.shape]
    S = graphs.synthetic_graph(a.shape, seed=0)
    X = torch.from_numpy(graphs.synthetic_features(a.shape, S.n, spec["features"], seed=1)).cuda()
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device="cuda")
    K = spec["hops"]
    ref = None
    times = {n: [] for n, _ in configs}
    try:
        for r in range(a.rounds + 1):
            order = configs if r % 2 == 0 else configs[::-1]
            for name, kv in order:
                for k in knobs:
                    _lib.check(lib.sgc_set_tuning(k.encode(), defaults[k]), "set_tuning")
                for k, v in kv:
                    _lib.check(lib.sgc_set_tuning(k.encode(), v), f"set_tuning {k}")
                out = propagate(csr, X, K)
                torch.cuda.synchronize()
                if ref is None:
                    ref = out.clone()
                if not torch.equal(out, ref):
                    raise SystemExit(f"config {name} changed the result")
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.steps):
                    propagate(csr, X, K)
                e.record()
                torch.cuda.synchronize()
                if r:
                    times[name].append(s.elapsed_time(e) / a.steps)
    finally:
        for k in knobs:
            lib.sgc_set_tuning(k.encode(), defaults[k])
    print(json.dumps({"shape": a.shape, "K": K, "bit_identical": True,
                      "median_ms": {n: float(np.median(t)) for n, t in times.items()},
                      "rounds_ms": {n: [round(v, 4) for v in t] for n, t in times.items()},
                      "configs": {n: dict(kv) for n, kv in configs}}), flush=True)


if __name__ == "__main__":
    main()
