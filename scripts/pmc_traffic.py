"""HBM traffic of the SpMM kernel from rocprofv3 PMC counters.

    # on the GPU box, one counter set per pass (gfx950 TCC slots: FETCH_SIZE
    # costs 3 of 4, WRITE_SIZE 2), kernel trace only beside the counters:
    cd /tmp && export TMPDIR=/tmp
    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d OUT/pmc_fetch -o p -- \
        python3 REPO/scripts/pmc_traffic.py workload
    rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d OUT/pmc_write -o p -- \
        python3 REPO/scripts/pmc_traffic.py workload
    rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d OUT/pmc_l2 -o p -- \
        python3 REPO/scripts/pmc_traffic.py workload
    python3 REPO/scripts/pmc_traffic.py summarize OUT      # -> profiles/pmc_reddit.json

Calibration (MI355X_MICROARCH.md, HBM section: FETCH_SIZE under-counts wide
coalesced reads on gfx950 and other widths are uncalibrated): the workload
first runs the SAME kernel over an identity S (N_cal rows, one nonzero each),
which reads every X row exactly once with the kernel's own dwordx2 gathers and
writes every Y row once -- a known byte count far beyond the 256 MiB
Infinity Cache.  read_factor = known_read_bytes / (FETCH_SIZE*1024) of that
launch is then applied to the Reddit-shape launches.
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

N_CAL = 1_000_000
F = 602
LD = 608     # X / Y row stride as propagate() lays them out: 128-B rows
LINES = (4 * F + 127) // 128  # 128-B lines one row's F floats touch (19)
REPEATS = 3


def workload():
    import numpy as np
    import torch

    from sgc_amd import graphs
    from sgc_amd.propagate import DeviceCSR, spmm
    dev = torch.device("cuda", 0)
    # calibration: identity S, X row i read once, Y row i written once
    rp = np.arange(N_CAL + 1, dtype=np.int32)
    ci = np.arange(N_CAL, dtype=np.int32)
    va = np.ones(N_CAL, dtype=np.float32)
    cal = DeviceCSR.from_host_arrays(rp, ci, va, device=dev)
    Xc = torch.randn((N_CAL, LD), device=dev)[:, :F]
    Yc = torch.empty((N_CAL, LD), device=dev)[:, :F]
    for _ in range(REPEATS):
        spmm(cal, Xc, out=Yc, use_plan=False)
    torch.cuda.synchronize()
    del Xc, Yc, cal
    from sgc_amd import _lib
    lib = _lib.load()
    for key in ("slice_floats", "max_vec"):
        v = os.environ.get("SGC_PMC_" + key.upper())
        if v is not None:
            lib.sgc_set_tuning(key.encode(), int(v))
    S = graphs.synthetic_graph("reddit", seed=0)
    X = torch.zeros((S.n, LD), device=dev)[:, :F]
    X.copy_(torch.from_numpy(graphs.synthetic_features("reddit", S.n, F, seed=1)))
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device=dev)
    Y = torch.empty((S.n, LD), device=dev)[:, :F]
    for _ in range(REPEATS):
        spmm(csr, X, out=Y)
    torch.cuda.synchronize()
    with open(os.environ.get("PMC_META", "/tmp/pmc_meta.json"), "w") as f:
        json.dump({"n": S.n, "nnz": S.nnz, "F": F, "n_cal": N_CAL}, f)
    print(f"pmc workload done: {S.nnz} nnz, tuning "
          f"{ {k: lib.sgc_get_tuning(k.encode()) for k in ('slice_floats', 'max_vec')} }")


def _rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    out = []
    for fn in files:
        with open(fn) as f:
            out.extend(csv.DictReader(f))
    return out


def _per_dispatch(rows, counter):
    """{dispatch_id: (kernel_name, grid_size, value)} summed over dimensions."""
    acc = {}
    for r in rows:
        if r.get("Counter_Name") != counter:
            continue
        k = int(r["Dispatch_Id"])
        name = r.get("Kernel_Name", "")
        grid = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
        v = float(r["Counter_Value"])
        if k in acc:
            acc[k] = (name, grid, acc[k][2] + v)
        else:
            acc[k] = (name, grid, v)
    return acc


def summarize(out_dir):
    n_cal, F_ = N_CAL, F
    tag = os.environ.get("SGC_PMC_TAG", "")
    fetch = _per_dispatch(_rows(os.path.join(out_dir, "pmc_fetch" + tag)), "FETCH_SIZE")
    write = _per_dispatch(_rows(os.path.join(out_dir, "pmc_write" + tag)), "WRITE_SIZE")
    l2 = _rows(os.path.join(out_dir, "pmc_l2" + tag))
    hit, miss = _per_dispatch(l2, "TCC_HIT_sum"), _per_dispatch(l2, "TCC_MISS_sum")

    def spmm_dispatches(d):
        """(calibration launches, Reddit-shape launches): main-kernel dispatch
        ids, each Reddit launch paired with the hub-kernel dispatches of the
        same sgc_spmm call (the hub rows' kernel runs beside the main one)."""
        ks = sorted(k for k, (nm, _, _) in d.items() if "spmm_csr_kernel" in nm)
        hubs = sorted(k for k, (nm, _, _) in d.items() if "spmm_hub_kernel" in nm)
        red = ks[REPEATS:2 * REPEATS]
        return ks[:REPEATS], [[k] + [h for h in hubs if prev < h < k]
                              for prev, k in zip([ks[REPEATS - 1]] + red[:-1], red)]

    cal_f, red_f = spmm_dispatches(fetch)
    cal_w, red_w = spmm_dispatches(write)
    cal_h, red_h = spmm_dispatches(hit)

    def mean(d, ks):  # ks: dispatch ids, or groups of ids summed per launch
        vals = [sum(d[j][2] for j in k) if isinstance(k, list) else d[k][2] for k in ks]
        return sum(vals) / max(1, len(vals))
    # line-granular: every X row touched once (LINES whole 128-B lines of its
    # 128-B aligned LD-float row), every Y row written once, plus the CSR
    known_read = 128 * LINES * n_cal + 4 * (n_cal + 1) + 8 * n_cal
    known_write = 128 * LINES * n_cal
    cal_fetch_b = mean(fetch, cal_f) * 1024
    cal_write_b = mean(write, cal_w) * 1024
    read_factor = known_read / cal_fetch_b
    write_factor = known_write / cal_write_b
    red_fetch_b = mean(fetch, red_f) * 1024 * read_factor
    red_write_b = mean(write, red_w) * 1024 * write_factor
    import math
    h, m = mean(hit, red_h), mean(miss, red_h)
    meta = {}
    try:
        meta = json.load(open(os.environ.get("PMC_META", "/tmp/pmc_meta.json")))
    except OSError:
        pass
    n, nnz = meta.get("n", 232965), meta.get("nnz", 23446803)
    alg = 4 * (n + 1) + 8 * nnz + 4 * F_ * nnz + 4 * F_ * n
    rec = {
        "workload": "reddit-shape spmm hop (232,965 rows, 23,446,803 nnz, F=602, X/Y ld 608 "
                    "as propagate() lays them out)",
        "hbm_bytes_per_launch": red_fetch_b + red_write_b,
        "hbm_read_bytes_per_launch": red_fetch_b,
        "hbm_write_bytes_per_launch": red_write_b,
        "raw_FETCH_SIZE_kB": mean(fetch, red_f), "raw_WRITE_SIZE_kB": mean(write, red_w),
        "calibration": {"kernel": "same spmm kernel over identity S, ld 608", "rows": n_cal,
                        "known_read_bytes": known_read, "known_write_bytes": known_write,
                        "FETCH_SIZE_bytes": cal_fetch_b, "WRITE_SIZE_bytes": cal_write_b,
                        "read_factor": read_factor, "write_factor": write_factor},
        "l2_hit_rate": h / (h + m) if (h + m) > 0 and not math.isnan(h) else None,
        "algorithmic_bytes_per_launch": alg,
        "compulsory_bytes_per_launch": 4 * (n + 1) + 8 * nnz + 8 * F_ * n,
        "traffic_over_algorithmic": (red_fetch_b + red_write_b) / alg,
    }
    rec["tuning"] = {k: os.environ.get("SGC_PMC_" + k.upper()) for k in ("slice_floats", "max_vec")}
    dst = os.path.join(ROOT, "profiles", f"pmc_reddit{tag}.json")
    with open(dst, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "workload":
        workload()
    else:
        summarize(sys.argv[2])
