"""Measured memory traffic of the SpMM hop from rocprofv3 PMC counters.

    # on the GPU box (scripts/pmc_session.sh runs these), one counter set per
    # pass (gfx950 TCC slots: FETCH_SIZE costs 3 of 4, WRITE_SIZE 2), kernel
    # trace only beside the counters:
    cd /tmp && export TMPDIR=/tmp
    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d OUT/pmc_fetch -o p -- \\
        python3 REPO/scripts/pmc_traffic.py workload SHAPE
    rocprofv3 --pmc WRITE_SIZE ... -d OUT/pmc_write ...
    rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum ... -d OUT/pmc_l2 ...
    python3 REPO/scripts/pmc_traffic.py summarize OUT SHAPE   # -> profiles/pmc_<shape>.json

The workload runs exactly what bench.py times: propagate() (K hops, X_0
re-laid into 128-B rows, ping-pong buffers, last hop into the caller's
[N, F] output) on the seeded BASELINE-shape graph, REPEATS times.  Every
SpMM launch (the light kernel + the spmm_hub_kernel dispatches of the same
call) is one "launch"; the JSON holds the mean bytes per launch.

Calibration (MI355X_MICROARCH.md, HBM section: FETCH_SIZE under-counts wide
coalesced reads on gfx950 and other widths are uncalibrated): the workload
first runs the SAME kernel over a random PERMUTATION S (N_cal rows, one
nonzero each, columns a seeded random permutation) at the shape's feature
width and row layout -- the gather pattern of the real hops, each X row read
exactly once in random order, each Y row written once: a known byte count
far beyond the 256 MiB Infinity Cache.  read_factor = known_read_bytes /
FETCH_SIZE bytes of that launch is then applied to the shape's launches.
The identity S (rows in order: a streaming pattern, the round-2
calibration) is run too and its factor reported beside it.  FETCH_SIZE counts Infinity-Cache hits (the guide), so the
result is the traffic beyond L2: an upper bound on HBM bytes.

The record carries the sha256 of the libsgc_amd.so it was taken with and the
tuning; bench.py refuses a record whose sha differs from the library it times.
"""
import csv
import glob
import hashlib
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

N_CAL = 1_000_000
REPEATS = 3
TUNING_KEYS = ("slice_floats", "max_vec", "hub_chunk", "heavy_pairs", "rows_per_wave")


def lib_sha():
    from sgc_amd import _lib
    with open(_lib.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def _meta_path(shape):
    return os.environ.get("PMC_META", f"/tmp/pmc_meta_{shape}.json")


def workload(shape):
    import numpy as np
    import torch

    from sgc_amd import _lib, graphs
    from sgc_amd.propagate import (SPMM_X_PADDED, SPMM_Y_PADDED, DeviceCSR, aligned_ld,
                                   column_groups_for, propagate, spmm)
    dev = torch.device("cuda", 0)
    spec = graphs.SHAPES[shape]
    F, K = spec["features"], spec["hops"]
    LD = aligned_ld(F)
    lib = _lib.load()
    for key in TUNING_KEYS:
        v = os.environ.get("SGC_PMC_" + key.upper())
        if v is not None:
            lib.sgc_set_tuning(key.encode(), int(v))
    # calibration: identity S (streaming), then a random permutation S (the
    # gather pattern); each X row read once, each Y row written once
    rp = np.arange(N_CAL + 1, dtype=np.int32)
    va = np.ones(N_CAL, dtype=np.float32)
    Xc = torch.randn((N_CAL, LD), device=dev)[:, :F]
    Yc = torch.empty((N_CAL, LD), device=dev)[:, :F]
    for ci in (np.arange(N_CAL, dtype=np.int32),
               np.random.default_rng(7).permutation(N_CAL).astype(np.int32)):
        cal = DeviceCSR.from_host_arrays(rp, ci, va, device=dev)
        for _ in range(REPEATS):  # the padded-buffer flags select the kernel the hops use
            spmm(cal, Xc, out=Yc, use_plan=False, flags=SPMM_X_PADDED | SPMM_Y_PADDED)
        torch.cuda.synchronize()
        del cal
    del Xc, Yc
    S = graphs.synthetic_graph(shape, seed=0)
    X0 = torch.from_numpy(graphs.synthetic_features(shape, S.n, F, seed=1)).to(dev)
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device=dev)
    out = torch.empty((S.n, F), device=dev)
    for _ in range(REPEATS):
        propagate(csr, X0, K, out=out)
    torch.cuda.synchronize()
    tuning = {k: int(lib.sgc_get_tuning(k.encode())) for k in TUNING_KEYS}
    with open(_meta_path(shape), "w") as f:
        json.dump({"shape": shape, "n": S.n, "nnz": S.nnz, "F": F, "K": K, "ld": LD,
                   "n_cal": N_CAL, "lib_sha256": lib_sha(), "tuning": tuning,
                   "groups": column_groups_for(csr, F)}, f)
    print(f"pmc workload done: {shape} {S.nnz} nnz, K={K}, tuning {tuning}")


def _rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    out = []
    for fn in files:
        with open(fn) as f:
            out.extend(csv.DictReader(f))
    return out


def _kernel_ms(d):
    """{dispatch_id: duration ms} from the kernel trace beside the counters."""
    out = {}
    for fn in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                try:
                    out[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) -
                                                  int(r["Start_Timestamp"])) * 1e-6
                except (KeyError, ValueError):
                    pass
    return out


def _per_dispatch(rows, counter):
    """{dispatch_id: (kernel_name, value)} summed over dimensions."""
    acc = {}
    for r in rows:
        if r.get("Counter_Name") != counter:
            continue
        k = int(r["Dispatch_Id"])
        v = float(r["Counter_Value"])
        name = r.get("Kernel_Name", "")
        acc[k] = (name, acc[k][1] + v) if k in acc else (name, v)
    return acc


def _launches(d, K, G=1):
    """(identity-calibration ids, permutation-calibration ids,
    [[main ids..., hub ids...] per hop]): a hop is G column-group dispatches
    of the light kernel and the hub dispatches among them."""
    ks = sorted(k for k, (nm, _) in d.items()
                if "spmm_csr_kernel" in nm or "spmm_rows_kernel" in nm)
    hubs = sorted(k for k, (nm, _) in d.items() if "spmm_hub_kernel" in nm)
    cal_id, cal_perm = ks[:REPEATS], ks[REPEATS:2 * REPEATS]
    main = ks[2 * REPEATS:2 * REPEATS + REPEATS * K * G]
    out, prev = [], cal_perm[-1]
    for i in range(0, len(main), G):
        grp = main[i:i + G]
        out.append(grp + [h for h in hubs if prev < h < grp[-1]])
        prev = grp[-1]
    return cal_id, cal_perm, out


def summarize(out_dir, shape):
    meta = json.load(open(_meta_path(shape)))
    K, F, LD, n_cal = meta["K"], meta["F"], meta["ld"], meta["n_cal"]
    n, nnz = meta["n"], meta["nnz"]
    fetch = _per_dispatch(_rows(os.path.join(out_dir, "pmc_fetch")), "FETCH_SIZE")
    write = _per_dispatch(_rows(os.path.join(out_dir, "pmc_write")), "WRITE_SIZE")
    l2 = _rows(os.path.join(out_dir, "pmc_l2"))
    hit, miss = _per_dispatch(l2, "TCC_HIT_sum"), _per_dispatch(l2, "TCC_MISS_sum")
    G = int(meta.get("groups", 1))
    calid_f, cal_f, red_f = _launches(fetch, K, G)
    calid_w, cal_w, red_w = _launches(write, K, G)
    _, _, red_h = _launches(hit, K, G)

    def mean(d, ks):
        vals = [sum(d[j][1] for j in k) if isinstance(k, list) else d[k][1] for k in ks]
        return sum(vals) / max(1, len(vals))
    lines = (4 * F + 127) // 128  # 128-B lines one row's F floats touch (aligned rows)
    known_read = 128 * lines * n_cal + 4 * (n_cal + 1) + 8 * n_cal
    known_write = 128 * lines * n_cal
    cal_fetch_b = mean(fetch, cal_f) * 1024
    cal_write_b = mean(write, cal_w) * 1024
    read_factor = known_read / cal_fetch_b
    write_factor = known_write / cal_write_b
    id_read_factor = known_read / (mean(fetch, calid_f) * 1024)
    id_write_factor = known_write / (mean(write, calid_w) * 1024)
    red_fetch_b = mean(fetch, red_f) * 1024 * read_factor
    red_write_b = mean(write, red_w) * 1024 * write_factor
    h, m = mean(hit, red_h), mean(miss, red_h)
    kms = _kernel_ms(os.path.join(out_dir, "pmc_fetch"))
    main_ms = [sum(kms[k] for k in g[:G]) for g in red_f if all(k in kms for k in g[:G])]
    names = sorted({fetch[g[0]][0] for g in red_f})
    # "void sgc::spmm_rows_kernel<16, 2, 16, true>(int const*, ...)" -> "spmm_rows_kernel<16, 2, 16, true>"
    kname = " / ".join(nm.split("(")[0].replace("void ", "").replace("sgc::", "") for nm in names)
    alg = 4 * (n + 1) + 8 * nnz + 4 * F * nnz + 4 * F * n
    comp = 4 * (n + 1) + 8 * nnz + 8 * F * n
    rec = {
        "workload": f"{shape}-shape propagate() K={K} ({n} rows, {nnz} nnz, F={F}; X_0 in 128-B rows "
                    f"to ld {LD}, intermediates ld {LD}, last hop into ld {F}), {REPEATS} times; "
                    f"one launch = one hop ({G} column-group dispatch(es) of {kname} + the "
                    f"spmm_hub_kernel dispatches among them)",
        "dispatches_per_launch": G,
        "light_kernel": kname,
        "lib_sha256": meta["lib_sha256"], "tuning": meta["tuning"],
        "hbm_bytes_per_launch": red_fetch_b + red_write_b,
        "hbm_read_bytes_per_launch": red_fetch_b,
        "hbm_write_bytes_per_launch": red_write_b,
        "raw_FETCH_SIZE_kB": mean(fetch, red_f), "raw_WRITE_SIZE_kB": mean(write, red_w),
        "calibration": {"kernel": f"same spmm kernel over a random permutation S (each X "
                                  f"row gathered once, random order), F={F}, ld {LD}",
                        "rows": n_cal, "known_read_bytes": known_read,
                        "known_write_bytes": known_write, "FETCH_SIZE_bytes": cal_fetch_b,
                        "WRITE_SIZE_bytes": cal_write_b, "read_factor": read_factor,
                        "write_factor": write_factor,
                        "identity_S_read_factor": id_read_factor,
                        "identity_S_write_factor": id_write_factor},
        "l2_hit_rate": h / (h + m) if (h + m) > 0 and not math.isnan(h) else None,
        "kernel_ms": (sum(main_ms) / len(main_ms)) if main_ms else None,
        "kernel_ms_note": f"{kname}: sum of a hop's {G} dispatch durations, mean over hops, in "
                          "the profiled FETCH_SIZE pass "
                          "(profiled passes run slower than unprofiled ones)",
        "algorithmic_bytes_per_launch": alg,
        "compulsory_bytes_per_launch": comp,
        "traffic_over_algorithmic": (red_fetch_b + red_write_b) / alg,
        "traffic_over_compulsory": (red_fetch_b + red_write_b) / comp,
        "launches": len(red_f),
    }
    dst = os.path.join(ROOT, "profiles", f"pmc_{shape}.json")
    with open(dst, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "workload":
        workload(sys.argv[2] if len(sys.argv) > 2 else "reddit")
    else:
        summarize(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "reddit")
