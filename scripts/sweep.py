"""Interleaved A/B timing of SpMM build variants and schedule thresholds in ONE
process (cdna_hip_programming.md 5.4 rule 24), Reddit-shape hop.

    python scripts/sweep.py [--libs a.so,b.so] [--thresholds 256,512,2048] [--rounds 8]

Every variant must stay bit-identical: the first output of each is compared
with the product library's.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from sgc_amd import _lib, graphs  # noqa: E402
from sgc_amd.propagate import DeviceCSR  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="")
    ap.add_argument("--thresholds", default="2048")
    ap.add_argument("--hubs", default="4096", help="hub thresholds (sgc_plan_build)")
    ap.add_argument("--slices", default="128", help="slice_floats values (sgc_set_tuning)")
    ap.add_argument("--vecs", default="4", help="max_vec values (sgc_set_tuning)")
    ap.add_argument("--knob", default="", help="one more sgc_set_tuning key: name=v1,v2")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--shape", default="reddit")
    ap.add_argument("--ld", default="0", help="X row strides to try (0 = F)")
    args = ap.parse_args()
    libs = [_lib.LIB_PATH] + [p for p in args.libs.split(",") if p]
    loaded = [(os.path.basename(p), _lib.load_path(p)) for p in libs]
    thresholds = [int(t) for t in args.thresholds.split(",")]

    dev = torch.device("cuda", 0)
    S = graphs.synthetic_graph(args.shape, seed=0)
    F = graphs.SHAPES[args.shape]["features"]
    X = torch.from_numpy(graphs.synthetic_features(args.shape, S.n, F, seed=1)).to(dev)
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device=dev)
    hubs = [int(x) for x in args.hubs.split(",")]
    plans = {(t, hb): csr.plan(0, S.n, t, hb) for t in thresholds for hb in hubs}
    Y = torch.empty_like(X)
    lds = [int(x) or F for x in args.ld.split(",")]
    Xs = {}
    for ld in lds:
        buf = torch.zeros((S.n, ld), device=dev)
        buf[:, :F] = X
        Xs[ld] = buf
    stream = _lib.stream_handle(dev)
    ref = None
    slices = [int(x) for x in args.slices.split(",")]
    vecs = [int(x) for x in args.vecs.split(",")]
    kname, kvals = (args.knob.split("=") + [""])[:2] if args.knob else ("", "")
    kvals = [int(x) for x in kvals.split(",")] if kname else [None]
    variants = [(f"{name}/v{mv}/s{sf}/ld{ld}/hub{hb}" + (f"/{kname}{kv}" if kname else ""), lib, t,
                 (sf, ld, hb, mv, kv)) for name, lib in loaded for t in thresholds for sf in slices
                for ld in lds for hb in hubs for mv in vecs for kv in kvals]

    def run(lib, t, cfg):
        sf, ld, hb, mv, kv = cfg
        lib.sgc_set_tuning(b"slice_floats", sf)
        lib.sgc_set_tuning(b"max_vec", mv)
        if kname and lib.sgc_set_tuning(kname.encode(), kv):
            raise RuntimeError(lib.sgc_last_error())
        pl = plans[(t, hb)]
        rc = lib.sgc_spmm_csr_f32(_lib.ptr(csr.row_ptr), _lib.ptr(csr.col_idx), _lib.ptr(csr.val),
                                  0, S.n, _lib.ptr(Xs[ld]), ld, _lib.ptr(Y), F, F, _lib.ptr(pl.rows),
                                  pl.n_heavy, pl.n_hub, pl.threshold, stream)
        if rc:
            raise RuntimeError(lib.sgc_last_error())

    times = {(n, t): [] for n, _, t, _ in variants}  # n encodes slice/ld/hub
    for name, lib, t, sf in variants:  # warm-up + correctness
        run(lib, t, sf)
        torch.cuda.synchronize()
        out = Y.cpu().numpy().view(np.uint32).copy()
        if ref is None:
            ref = out
        elif not np.array_equal(ref, out):
            raise SystemExit(f"variant {name} t={t} is NOT bit-identical")
    for _ in range(args.rounds):
        for name, lib, t, sf in variants:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.reps):
                run(lib, t, sf)
            e.record()
            e.synchronize()
            times[(name, t)].append(s.elapsed_time(e) / args.reps)
    alg = 4 * (S.n + 1) + 8 * S.nnz + 4 * F * S.nnz + 4 * F * S.n
    res = []
    for (name, t), v in times.items():
        med = float(np.median(v))
        res.append({"lib": name, "threshold": t, "median_ms": round(med, 4),
                    "min_ms": round(float(np.min(v)), 4), "gather_model_TBps": round(alg / med / 1e9, 3)})
    res.sort(key=lambda r: r["median_ms"])
    for r in res:
        print(json.dumps(r))


if __name__ == "__main__":
    del ctypes
    main()
