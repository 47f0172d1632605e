"""Interleaved A/B timing of SpMM build variants on the launch shapes the
multi-GPU paths issue: feature groups / blocks of W floats over all rows or a
1/P row block (Reddit shape).  One process, rounds interleaved
(cdna_hip_programming.md 5.4 rule 24); every variant is checked bit-identical
to the product library on each case.

    python scripts/sweep_narrow.py --libs a.so,b.so --widths 128,224,602 --parts 1,8
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from sgc_amd import _lib, graphs  # noqa: E402
from sgc_amd.distributed import equal_row_bounds  # noqa: E402
from sgc_amd.propagate import DeviceCSR  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="")
    ap.add_argument("--widths", default="128,224,602")
    ap.add_argument("--parts", default="1,8")
    ap.add_argument("--max-vec", default="4")
    ap.add_argument("--hub-chunk", default="0")
    ap.add_argument("--hub-priority", default="0")
    ap.add_argument("--slices", default="128", help="slice_floats values")
    ap.add_argument("--heavy-packed", default="0", help="heavy_packed values")
    ap.add_argument("--hubs", default="auto", help="hub thresholds per case ('auto' = default)")
    ap.add_argument("--heavies", default="default", help="heavy-row thresholds per case")
    ap.add_argument("--shape", default="reddit")
    ap.add_argument("--unaligned", action="store_true",
                    help="also read each width straight from the [N, 602] input (ld 602)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    libs = [_lib.LIB_PATH] + [p for p in args.libs.split(",") if p]
    loaded = [(os.path.basename(p), _lib.load_path(p)) for p in libs]
    dev = torch.device("cuda", 0)
    S = graphs.synthetic_graph(args.shape, seed=0)
    F = graphs.SHAPES[args.shape]["features"]
    X = torch.from_numpy(graphs.synthetic_features(args.shape, S.n, F, seed=1)).to(dev)
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device=dev)
    rp = np.asarray(S.row_ptr, dtype=np.int64)
    stream = _lib.stream_handle(dev)
    cases = []
    widths = [F if x == "F" else int(x) for x in args.widths.split(",")]
    for w in widths:
        ld = (w + 31) // 32 * 32
        Xw = torch.zeros((S.n, ld), device=dev)
        Xw[:, :w] = X[:, :w]
        for P in (int(x) for x in args.parts.split(",")):
            r0, r1 = 0, int(equal_row_bounds(S.n, P)[1])
            Y = torch.empty((r1 - r0, ld), device=dev)
            nz = int(rp[r1] - rp[r0])
            gb = (4 * (r1 - r0 + 1) + 8 * nz + 4 * w * nz + 4 * w * (r1 - r0)) / 1e9
            for hv in args.heavies.split(","):
                th = None if hv == "default" else int(hv)
                for hb in args.hubs.split(","):
                    pl = csr.plan(r0, r1, th, None if hb == "auto" else int(hb), w)
                    name = f"w{w}/P{P}/heavy{hv}:{pl.n_heavy}/hub{hb}:{pl.n_hub}"
                    cases.append((name, Xw, ld, w, r0, r1, pl, Y, gb))
                    if args.unaligned:
                        cases.append((name + f"/ld{F}", X, F, w, r0, r1, pl, Y, gb))
    mvs = [int(x) for x in args.max_vec.split(",")]
    hcs = [int(x) for x in args.hub_chunk.split(",")]
    hps = [int(x) for x in args.hub_priority.split(",")]
    sfs = [int(x) for x in args.slices.split(",")]
    hks = [int(x) for x in args.heavy_packed.split(",")]
    variants = [(f"{name}/hc{hc}/hp{hp}/s{sf}/pk{pk}", lib, (mv, hc, hp, sf, pk))
                for name, lib in loaded
                for mv in mvs for hc in hcs for hp in hps for sf in sfs for pk in hks]

    def run(lib, cfg, c):
        mv, hc, hp, sf, pk = cfg
        lib.sgc_set_tuning(b"slice_floats", sf)
        lib.sgc_set_tuning(b"heavy_packed", pk)
        _, Xw, ld, w, r0, r1, pl, Y, _ = c
        lib.sgc_set_tuning(b"max_vec", mv)
        lib.sgc_set_tuning(b"hub_chunk", hc)
        lib.sgc_set_tuning(b"hub_priority", hp)
        rc = lib.sgc_spmm_csr_f32(_lib.ptr(csr.row_ptr), _lib.ptr(csr.col_idx), _lib.ptr(csr.val),
                                  r0, r1, _lib.ptr(Xw), ld, _lib.ptr(Y), Y.stride(0), w,
                                  _lib.ptr(pl.rows),
                                  pl.n_heavy, pl.n_hub, pl.threshold, stream)
        if rc:
            raise RuntimeError(lib.sgc_last_error())

    for c in cases:
        ref = None
        for name, lib, mv in variants:
            run(lib, mv, c)
            torch.cuda.synchronize()
            out = c[7][:, :c[3]].cpu().numpy().view(np.uint32).copy()
            if ref is None:
                ref = out
            elif not np.array_equal(ref, out):
                raise SystemExit(f"variant {name} cfg={mv} case {c[0]} is NOT bit-identical")
    times = {(c[0], v[0], v[2]): [] for c in cases for v in variants}
    for _ in range(args.rounds):
        for c in cases:
            for name, lib, mv in variants:
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(args.reps):
                    run(lib, mv, c)
                e.record()
                e.synchronize()
                times[(c[0], name, mv)].append(s.elapsed_time(e) / args.reps)
    gbs = {c[0]: c[8] for c in cases}
    for (case, name, mv), v in sorted(times.items()):
        med = float(np.median(v))
        print(json.dumps({"case": case, "lib": name, "max_vec": mv[0], "median_ms": round(med, 4),
                          "gather_model_TBps": round(gbs[case] / med, 3)}), flush=True)


if __name__ == "__main__":
    main()
