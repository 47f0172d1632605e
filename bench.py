"""bench.py -- SGC propagation hot path on MI355X: propagated edges/s.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--shape reddit]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

`bench.py --gpus N` (N > 1) without torchrun's environment launches its own N
ranks (a torch.distributed.run child, started before anything touches the
GPU) and relays rank 0's line; its exit status is non-zero if any rank fails.
N = 1 times the public call itself, sgc_precompute(features, adj, K).

Metric (BASELINE.json): propagated edges/s = hops * nnz(S) / t, where t is
one sgc_precompute (all K hops of S.X, reference utils.py:92-97) over the
synthetic Reddit-shape graph (232,965 nodes, 11,606,919 undirected edges,
nnz(S) = 23,446,803, F = 602, K = 2), inputs resident in HBM.
A "step" = one full K-hop propagation.  N > 1: `value` times the SAME call
as N = 1 -- sgc_precompute(features, adj, K) on every rank under the process
group (sgc_amd.multigpu: every rank gets the whole X_K, as the reference
returns it; partition SGC_AMD_PARTITION, default "auto": the first call times
replicate / features / lines on the node, max over ranks, and keeps the
fastest -- `config.partition` names it, `config.auto_seconds` lists the
times); total work fixed, so scaling is "strong".  Beside it (`sharded_output`) the
partitioned propagator with sharded output (sgc_amd.distributed):
  --partition rows  S row-partitioned (nnz-balanced row blocks, SURVEY.md
                8(e)); RCCL all-gather of X_k after each hop that feeds another,
                optionally pipelined in feature groups, hub rows on their own streams
  --partition tiles  R x C: row blocks x --col-blocks feature blocks; the
                per-hop all-gather runs within each feature block's R ranks
  --partition cyclic  row tiles dealt round-robin; each all-gather carries one
                column group (--cyclic-groups G) and the next hop consumes it
                as it arrives (column-group passes, SGC_SPMM_ACCUMULATE)
  --partition features  each rank runs all K hops on its block of feature
                columns over the full S, no exchange between hops; sharded
                output by one all-to-all of the row blocks of X_K
  --partition auto (default)  rows vs cyclic vs features (vs tiles), timed
                on the node (max over ranks); the fastest is kept

Also printed (same JSON line, N = 1):
  roofline      the SpMM hop (spmm_rows_kernel / spmm_csr_kernel, joined with
                spmm_hub_kernel on its side stream), timed with the library's
                HIP events on the launch stream (sgc_timing_*, each kernel also
                on its own stream) over a second run of the same steps right
                after the timed one (the events cost host time per launch:
                `value` is taken without them, ms_per_step_instrumented shows
                the difference).  achieved = MEASURED bytes per launch
                (rocprofv3 FETCH_SIZE + WRITE_SIZE, calibrated, from
                profiles/pmc_<shape>.json -- used only when its recorded
                libsgc_amd.so sha256 equals the library being timed) / the
                mean hop time; frac = achieved / 8 TB/s.  Beside it the two
                byte MODELS of SURVEY.md 8(d): the gather model (every
                nonzero re-reads its X row; no cache reuse; an upper bound
                that exceeds the HBM peak when the live X slice is
                cache-resident) and the compulsory model (S, X and Y once).
  shapes        the same measurement for the other BASELINE configs
                (Cora-, Pubmed-, RMAT-shape), rank 0 at N = 1
  classifier    the SGC classifier at Reddit-train shape (152,410 x 602 -> 41):
                the MFMA forward and weight backward with bytes and frac, the
                reference's training closure (drop-in SGC vs nn.Linear vs the
                fused loss) and reddit.py's 2-step LBFGS (sgc_amd.classifier_bench)
  cpu_baseline  the reference's arithmetic as written -- torch.spmm(COO, X)
                (utils.py:95), median of 3 hops on this host; plus torch CSR
                and this library's own CPU twin at every available core
"""
import argparse
import hashlib
import json
import os
import platform
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from sgc_amd import graphs  # noqa: E402
from sgc_amd.propagate import DeviceCSR, collect_launch_timing, kernel_timing  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
BASELINE_METRIC = ("propagated edges/sec (K-hop SpMM) + precompute wall-time, "
                   "Reddit K=2 at 1/2/4/8 GPUs")
SUB_STEPS = {"cora": (20, 5), "pubmed": (20, 5), "reddit": (10, 3), "rmat": (3, 1)}


def output_check(shape, K, Y, seed):
    """{"output_sha_ok": bool | None, ...}: SHA-256 of one timed call's X_K
    against the hash the reference's own sgc_precompute produced for the
    same seeded graph and features (tests/golden/shapes.json, written by
    tests/golden/gen_golden.py).  None when no golden covers (shape, K, seed)."""
    rec = {"output_sha_ok": None, "output_sha_basis": None}
    try:
        with open(os.path.join(ROOT, "tests", "golden", "shapes.json")) as f:
            g = json.load(f).get(shape)
    except (OSError, ValueError):
        g = None
    if not g or str(K) not in g.get("outputs", {}) or g.get("seed") != seed or \
            g.get("feature_seed") != seed + 1:
        rec["output_sha_basis"] = f"no golden for {shape} K={K} seed={seed}"
        return rec
    h = hashlib.sha256()
    Yc = Y.detach()
    rows = max(1, (256 << 20) // max(1, 4 * Yc.shape[1]))  # 256 MB host chunks
    for r in range(0, Yc.shape[0], rows):
        h.update(np.ascontiguousarray(Yc[r:r + rows].cpu().numpy()).tobytes())
    got = h.hexdigest()
    rec["output_sha_ok"] = got == g["outputs"][str(K)]["sha"]
    rec["output_sha_basis"] = ("sha256 of the last timed call's X_K vs tests/golden/shapes.json "
                               f"[{shape}][outputs][{K}] (the reference's sgc_precompute)")
    if not rec["output_sha_ok"]:
        rec["output_sha"] = got
    return rec


def gather_model_bytes(n, nnz, F):
    """row_ptr + (col, val) + one X row per nonzero + Y."""
    return 4 * (n + 1) + 8 * nnz + 4 * F * nnz + 4 * F * n


def compulsory_bytes(n, nnz, F):
    """S once, X once, Y once."""
    return 4 * (n + 1) + 8 * nnz + 8 * F * n


def lib_sha256():
    from sgc_amd import _lib
    h = hashlib.sha256()
    with open(_lib.LIB_PATH, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def host_cores():
    """(cores this process may use, how that was decided): the affinity mask,
    bounded by a cgroup CPU quota when one is set."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    how = f"sched_getaffinity={n}"
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            q = max(1, int(int(quota) / int(period)))
            how += f", cgroup cpu.max quota={q}"
            n = min(n, q)
    except (OSError, ValueError):
        pass
    return max(1, n), how


def cpu_baseline(S, X_host, reps=3):
    """The reference's arithmetic on this host: torch.spmm(COO, X) -- what
    utils.py:95 runs each hop -- median of `reps` full hops after a warm-up
    hop on 64 feature columns (allocator first touch).  aten's COO kernel is
    single-threaded whatever torch.get_num_threads() says, so
    cores = 1.  Beside it, at every available core: torch CSR
    (torch.sparse.mm, bit-identical output, the best CPU torch path) and this
    library's own CPU twin (sgc_propagate_f32_cpu, bit-identical)."""
    from sgc_amd.propagate import DeviceCSR as _CSR
    from sgc_amd.propagate import propagate as _prop
    rows, cols, vals = S.coo()
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.stack([rows, cols])),
                                  torch.from_numpy(vals), (S.n, S.n))
    X = torch.from_numpy(X_host)
    torch.spmm(adj, X[:, :64].contiguous())
    t_coo = []
    for _ in range(reps):
        t0 = time.perf_counter()
        torch.spmm(adj, X)
        t_coo.append(time.perf_counter() - t0)
    med = float(np.median(t_coo))
    cores, how = host_cores()
    rec = {"value": S.nnz / med, "unit": "edges/s", "cores": 1, "kind": "reference",
           "sample": f"1 hop of torch.spmm(COO fp32 {S.n}x{S.n}, nnz {S.nnz}; X [{S.n},"
                     f"{X.shape[1]}]) = reference utils.py:95 as written; median of {reps} hops "
                     f"after a 64-column warm-up: {med:.2f} s (aten's COO kernel is single-"
                     f"threaded)",
           "coo_seconds": [round(t, 3) for t in t_coo],
           "host_cpu": cpu_model(), "os_cpu_count": os.cpu_count(),
           "host_cores_available": cores, "host_cores_rule": how}
    saved = torch.get_num_threads()
    torch.set_num_threads(cores)
    try:
        csr = adj.to_sparse_csr()
        torch.sparse.mm(csr, X)
        t_csr = []
        for _ in range(reps):
            t0 = time.perf_counter()
            torch.sparse.mm(csr, X)
            t_csr.append(time.perf_counter() - t0)
        m = float(np.median(t_csr))
        rec["csr_all_cores"] = {"value": S.nnz / m, "unit": "edges/s", "cores": cores,
                                "seconds_median": round(m, 4),
                                "what": "torch.sparse.mm(adj.to_sparse_csr(), X), one hop"}
        hc = _CSR._from_torch_cpu(adj)
        out = torch.empty_like(X)
        _prop(hc, X, 1, out=out)
        t_tw = []
        for _ in range(reps):
            t0 = time.perf_counter()
            _prop(hc, X, 1, out=out)
            t_tw.append(time.perf_counter() - t0)
        m = float(np.median(t_tw))
        rec["cpu_twin_all_cores"] = {"value": S.nnz / m, "unit": "edges/s", "cores": cores,
                                     "seconds_median": round(m, 4),
                                     "what": "this library's CPU twin sgc_propagate_f32_cpu, "
                                             "one hop (bit-identical to the reference)"}
    finally:
        torch.set_num_threads(saved)
    return rec


def load_traffic(shape, lib_sha, groups=1):
    """Measured bytes per hop from profiles/pmc_<shape>.json, or (None, why)
    when absent or taken on a different build of the library or schedule
    (column-group dispatches per hop)."""
    p = os.path.join(ROOT, "profiles", f"pmc_{shape}.json")
    if not os.path.exists(p):
        return None, f"no {os.path.relpath(p, ROOT)}"
    with open(p) as f:
        d = json.load(f)
    if d.get("lib_sha256") != lib_sha:
        return None, (f"{os.path.relpath(p, ROOT)} was taken on libsgc_amd.so "
                      f"{str(d.get('lib_sha256'))[:12]}, not the timed {lib_sha[:12]}: refused")
    if int(d.get("dispatches_per_launch", 1)) != int(groups):
        return None, (f"{os.path.relpath(p, ROOT)} counts {d.get('dispatches_per_launch', 1)} "
                      f"dispatch(es) per hop, the timed schedule {groups}: refused")
    return d, os.path.relpath(p, ROOT)


def roofline(shape, n, nnz, F, hop_ms, light_ms, hub_ms, lib_sha, launch_desc, light_kernel,
             groups=1, light_dispatch_ms=None):
    gm = gather_model_bytes(n, nnz, F)
    cb = compulsory_bytes(n, nnz, F)
    t = hop_ms * 1e-3
    pmc, src = load_traffic(shape, lib_sha, groups)
    rec = {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "kernel": (f"{light_kernel} (+ spmm_hub_kernel beside it, joined)" if hub_ms else
                      str(light_kernel)),
           "kernel_mean_ms": hop_ms, "launch_unit": launch_desc,
           "light_kernel_mean_ms": light_ms, "hub_kernel_mean_ms": hub_ms,
           "dispatches_per_launch": groups,
           "light_kernel_dispatch_mean_ms": light_dispatch_ms,
           "hub_tail_ms": (max(0.0, hub_ms - light_ms) if hub_ms is not None and light_ms
                           else None),
           "gather_model_bytes_per_launch": gm,
           "gather_model_frac": gm / t / 1e9 / HBM_PEAK_GBS,
           "compulsory_bytes_per_launch": cb,
           "compulsory_frac": cb / t / 1e9 / HBM_PEAK_GBS,
           "traffic_source": src}
    if pmc is not None:
        traffic = pmc["hbm_bytes_per_launch"]
        rec.update({"achieved": traffic / t / 1e9, "frac": traffic / t / 1e9 / HBM_PEAK_GBS,
                    "traffic": traffic, "achieved_basis": "measured (PMC FETCH_SIZE+WRITE_SIZE, "
                    "calibrated; counts Infinity-Cache hits, so an upper bound on HBM bytes)",
                    "l2_hit_rate": pmc.get("l2_hit_rate"),
                    "pmc_kernel_ms": pmc.get("kernel_ms")})
    else:
        rec.update({"achieved": cb / t / 1e9, "frac": cb / t / 1e9 / HBM_PEAK_GBS,
                    "traffic": None, "achieved_basis": "compulsory bytes (no matching PMC file)"})
    return rec


class LaunchTimer:
    """The library's own per-launch HIP events (sgc_timing_*) over the timed
    region: each SpMM launch's light-kernel and hub-kernel durations, each on
    the stream it runs on, and its span as the launch stream sees it (hub
    kernel joined) -- the hop time of the roofline."""

    def __init__(self, groups=1):
        self.groups = max(1, int(groups))  # dispatches per hop (column groups)
        self.dispatch_light = []

    def start(self):
        collect_launch_timing()  # drop anything recorded before
        kernel_timing(True)

    def stop(self):
        kernel_timing(False)
        torch.cuda.synchronize()
        light, hub, span, kind = collect_launch_timing()
        names = [k for k in kind if k]
        top = max(set(names), key=names.count) if names else None
        self.dispatch_light = list(light)
        G = self.groups
        if G > 1:  # a hop = G consecutive launches on one stream: sum them
            def per_hop(v):
                return [sum(x or 0.0 for x in v[i:i + G]) for i in range(0, len(v) - G + 1, G)]
            has_hub = any(h is not None for h in hub)
            span, light = per_hop(span), per_hop(light)
            hub = per_hop(hub) if has_hub else []
        return span, light, [h for h in hub if h is not None], top


def mean_or_none(v):
    return float(np.mean(v)) if v else None


def timed(step, steps, warmup, distributed, dev, on_start=None, on_stop=None, events=True):
    """W untimed warm-ups, then exactly `steps` steps between
    synchronise + barrier pairs; returns (max-over-ranks elapsed s, per-step
    ms from events on the current stream -- [] with events=False: the value
    run takes no per-step events, which cost host time per step that a
    Pubmed-shape call (~0.1 ms) would otherwise carry)."""
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    if on_start:
        on_start()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(steps)] if events else []
    t0 = time.perf_counter()
    if events:
        for s, e in evs:
            s.record()
            step()
            e.record()
    else:
        for _ in range(steps):
            step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    extra = on_stop() if on_stop else None
    step_ms = [s.elapsed_time(e) for s, e in evs]
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    return elapsed, step_ms, extra


def single_gpu_shape(shape, args, dev, lib_sha, steps, warmup, S=None, X_host=None, K=None):
    """One BASELINE config on one GPU through the public call itself --
    sgc_precompute(features, adj, K), reference utils.py:92-97, on a torch COO
    adjacency whose CSR it caches on the first call (as reddit.py's repeated
    calls would) -- throughput, per-kernel times, roofline and the first-call
    (ingest + plan + propagation) time."""
    import importlib
    prop_mod = importlib.import_module("sgc_amd.propagate")
    from sgc_amd.utils import sgc_precompute
    if args.threshold is not None:
        prop_mod.DEFAULT_HEAVY_THRESHOLD = args.threshold
    if args.hub_threshold is not None:
        prop_mod.DEFAULT_HUB_THRESHOLD = args.hub_threshold
    spec = graphs.SHAPES[shape]
    K = K or spec["hops"]
    t_gen = time.perf_counter()
    if S is None:
        S = graphs.synthetic_graph(shape, seed=args.seed)
        X_host = graphs.synthetic_features(shape, S.n, spec["features"], seed=args.seed + 1)
    t_gen = time.perf_counter() - t_gen
    n, F, nnz = S.n, X_host.shape[1], S.nnz
    X0 = torch.from_numpy(X_host).to(dev)
    # first call on a fresh torch COO adjacency (reference layout, utils.py:23-30):
    # ingest (COO -> CSR) + plan + K hops, as sgc_precompute's first call pays it
    rows, cols, vals = S.coo()
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.stack([rows, cols])),
                                  torch.from_numpy(vals), (n, n)).to(dev)
    del rows, cols, vals
    torch.cuda.synchronize()
    # what the drop-in loaders do when they move the data to the GPU
    # (load_reddit_data / load_citation: the code objects load there, once
    # per process), then the reference's first, timed call (reddit.py:43)
    warm_s = prop_mod.warmup(dev)
    _, first_s = sgc_precompute(X0, adj, K)
    ingest_s = adj._sgc_amd_csr[1].ingest_seconds
    groups = prop_mod.column_groups_for(adj._sgc_amd_csr[1], F)
    launches = LaunchTimer(groups)

    last = [None]

    def step():  # the public call, as the reference's drivers make it
        last[0] = sgc_precompute(X0, adj, K)[0]

    # value: the call as a caller sees it, nothing else in the loop; then the
    # same number of steps again with the library's per-launch events on (the
    # roofline's kernel times) -- at Cora shape those events alone would add
    # more host time per step than the two hops take on the GPU
    elapsed, _, _ = timed(step, steps, warmup, False, dev, events=False)
    check = output_check(shape, K, last[0], args.seed)  # the last timed call's X_K
    last[0] = None
    elapsed_i, step_ms, (hop_ms, light, hub, kernel) = timed(
        step, steps, 1, False, dev, on_start=launches.start, on_stop=launches.stop)
    hop_mean = float(np.mean(hop_ms))
    rec = {"value": K * nnz * steps / elapsed, "unit": "edges/s",
           "ms_per_step": elapsed * 1e3 / steps,
           "ms_per_step_median": float(np.median(step_ms)),
           "ms_per_step_median_basis": "per-step events of the instrumented run",
           "ms_per_step_events": [round(v, 4) for v in step_ms],
           "ms_per_step_instrumented": elapsed_i * 1e3 / steps,
           "steps": steps, "warmup": warmup,
           "config": {"workload": f"{shape}-shape sgc_precompute K={K}", "nodes": n,
                      "undirected_edges": spec["edges"], "nnz": nnz, "features": F, "hops": K},
           "first_call_seconds": round(first_s, 4), "ingest_seconds": round(ingest_s, 4),
           "loader_warmup_seconds": round(warm_s, 4),
           "generate_seconds": round(t_gen, 2),
           "roofline": roofline(shape, n, nnz, F, hop_mean, mean_or_none(light),
                                mean_or_none(hub), lib_sha,
                                f"one hop over all {n} rows" + (
                                    f" = {groups} column-group dispatches" if groups > 1 else ""),
                                kernel, groups, mean_or_none(launches.dispatch_light)),
           "hop_ms_median": float(np.median(hop_ms)),
           "timed_call": "sgc_precompute(features, adj, K) (sgc_amd.utils, the drop-in)"}
    rec.update(check)
    del X0, adj
    torch.cuda.empty_cache()
    return rec, S, X_host


def build_dist_step(args, S, X0, dev, rank, world, K, output, timing):
    """(step, parallelism, launch description) for the N > 1 path.  While
    timing["on"], every SpMM launch is bracketed by events on its stream and
    its compulsory bytes (its rows of S, the X columns it reads once, its Y)
    are recorded."""
    n, F = X0.shape
    tp = None

    def bracket(fn, nbytes):
        def run(*a, **k):
            if not timing["on"] or "hub" in a[3:]:  # time the light launches (rank 0's rows)
                return fn(*a, **k)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            r = fn(*a, **k)
            e.record()
            timing["pairs"].append((s, e))
            timing["bytes"].append(nbytes(*a))
            return r
        return run

    backend = "rccl" if args.dist_backend == "nccl" else "gloo rehearsal"
    staging = args.dist_backend == "gloo"
    if args.partition == "features":
        from sgc_amd.distributed import FeaturePartitionedPropagator, feature_bounds
        from sgc_amd.propagate import spmm as spmm_hip
        csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device=dev)
        rp = np.asarray(S.row_ptr, dtype=np.int64)

        def launch_bytes(X, r0, r1, out):
            nz, w = int(rp[r1] - rp[r0]), X.shape[1]
            return 4 * (r1 - r0 + 1) + 8 * nz + 4 * w * n + 4 * w * (r1 - r0)

        prop = FeaturePartitionedPropagator(
            csr, rank=rank, world_size=world,
            spmm_fn=bracket(lambda X, r0, r1, out: spmm_hip(
                csr, X, r0, r1, out=out, threshold=args.threshold,
                hub_threshold=args.hub_threshold), launch_bytes),
            chunks=args.chunks, host_staging=staging, exchange=args.exchange)
        fb, fB = feature_bounds(F, world)
        pairwise = args.exchange == "pairwise" or (args.exchange == "auto" and world == 2)
        exch = ((f"a pairwise exchange of the row blocks of X_K overlapped with the last hop "
                 f"({prop._pieces(world)} piece(s) per destination)" if pairwise else
                 "one all-to-all of the row blocks of X_K") if output == "sharded" else
                f"one all-gather of X_K pipelined with the last hop in {args.chunks} row chunks")
        par = (f"feature-partition x{world} ({fB}-column blocks, all K hops local) + {backend} "
               f"{exch}; output {output}")
        unit = f"rank 0's SpMM launches, {int(fb[1] - fb[0])} feature columns"
    elif args.partition == "lines":
        from sgc_amd.distributed import (LinePartitionedPropagator, _default_spmm, line_bounds,
                                         make_shard)
        from sgc_amd.propagate import spmm as spmm_hip
        csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device=dev)
        rp = np.asarray(S.row_ptr, dtype=np.int64)
        shard = make_shard(S.row_ptr, S.col_idx, S.val, rank, world, dev)

        def main_bytes(X, r0, r1, out, flags=0):
            nz, w = int(rp[r1] - rp[r0]), X.shape[1]
            return 4 * (r1 - r0 + 1) + 8 * nz + 4 * w * n + 4 * w * (r1 - r0)

        def tail_bytes(sh, X, out, *rest):
            w = X.shape[1]
            return 4 * (sh.rows + 1) + 8 * sh.nnz + 4 * w * n + 4 * w * sh.rows

        prop = LinePartitionedPropagator(
            shard, csr=csr,
            main_spmm_fn=bracket(lambda X, r0, r1, out, flags=0: spmm_hip(
                csr, X, r0, r1, out=out, flags=flags, threshold=args.threshold,
                hub_threshold=args.hub_threshold), main_bytes),
            tail_spmm_fn=bracket(_default_spmm, tail_bytes),
            chunks=args.chunks, host_staging=staging)
        prop._padded_ok = True  # the bracketed engine launches take the pad flags
        W, T = line_bounds(F, world)
        exch = ("one all-to-all of the main blocks' rows of X_K" if output == "sharded" else
                f"one all-gather of X_K pipelined with the last hop in {args.chunks} row chunks")
        par = (f"line-partition x{world} ({W}-column line blocks over all rows, all K hops "
               f"local; the {F - T} tail columns by nnz-balanced row blocks, all-gathered after "
               f"each hop on a tail stream) + {backend} {exch}; output {output}")
        unit = f"rank 0's SpMM launches ({W}-column main block + its tail rows)"
    elif args.partition == "cyclic":
        from sgc_amd.distributed import CyclicRowPropagator, _cyclic_spmm

        def launch_bytes(csr, X, out, rows, acc=False, part="all", thresholds=None):
            r0, r1 = rows
            w = X.shape[1]
            nz = csr.range_nnz(r0, r1)
            return (4 * (r1 - r0 + 1) + 8 * nz + 4 * w * min(X.shape[0], nz) +
                    4 * w * (r1 - r0) * (2 if acc else 1))

        groups = args.cyclic_groups or (1 if world <= 2 else 2 if world <= 4 else 3)
        prop = CyclicRowPropagator(S.row_ptr, S.col_idx, S.val, rank, world, dev,
                                   tile=args.cyclic_tile, groups=groups,
                                   host_staging=staging,
                                   spmm_fn=bracket(_cyclic_spmm, launch_bytes))
        sh = prop.shard
        exch = ("all-gathers of X_k after each hop but the last" if output == "sharded" else
                "all-gathers of X_k after every hop")
        par = (f"cyclic row tiles x{world} ({sh.tile}-row tiles round-robin) + {backend} {exch}, "
               f"{sh.groups} per hop, each one column group, consumed as it arrives by "
               f"column-group passes (SGC_SPMM_ACCUMULATE); output {output}")
        unit = (f"rank 0's SpMM launches ({sh.n_valid} rows, {sh.nnz} nnz, "
                f"{sh.groups} row chunks / column-group passes per hop)")
    else:
        from sgc_amd.distributed import (RowPartitionedPropagator, TiledPropagator,
                                         _default_spmm, feature_bounds, make_shard)

        def launch_bytes(sh, X, out, *rest):
            w = X.shape[1]
            return 4 * (sh.rows + 1) + 8 * sh.nnz + 4 * w * n + 4 * w * sh.rows

        C = args.col_blocks if args.partition == "tiles" else 1
        auto = args.group_floats == "auto"
        gf0 = 0 if auto else int(args.group_floats)
        spmm_fn = bracket(_default_spmm, launch_bytes)
        if C > 1:
            if output != "sharded":
                raise SystemExit("--partition tiles: output sharded only")
            tp = TiledPropagator(S.row_ptr, S.col_idx, S.val, rank, world, C, dev,
                                 group_floats=gf0, host_staging=staging, spmm_fn=spmm_fn)
            prop, shard = tp.prop, tp.shard
            fb, _ = feature_bounds(F, C)
            Xa = X0[:, int(fb[tp.j]):int(fb[tp.j + 1])]
        else:
            shard = make_shard(S.row_ptr, S.col_idx, S.val, rank, world, dev)
            prop = RowPartitionedPropagator(shard, spmm_fn=spmm_fn, group_floats=gf0,
                                            host_staging=staging)
            Xa = X0
        tuned = ""
        if auto and shard.world_size > 1:  # untimed setup, like the plans
            tt = prop.autotune(Xa, K, output="sharded" if C > 1 else output)
            tuned = " (autotuned: " + ", ".join(f"{g}: {t * 1e3:.2f} ms"
                                                for g, t in tt.items()) + ")"
        gf = prop.group_floats
        exch = ("all-gather of X_k after each hop but the last" if output == "sharded" else
                "all-gather of X_k after every hop")
        if C > 1:
            par = (f"2-D tiles {world // C} nnz-balanced row blocks x {C} feature blocks + "
                   f"{backend} {exch} within each feature block's {world // C} ranks, pipelined "
                   f"in {gf}-float groups{tuned}, + one all-gather of the {C} tiles of each row "
                   f"block; output sharded")
        else:
            par = (f"row-partition x{world} (nnz-balanced row blocks) + {backend} {exch}, "
                   f"pipelined in {gf}-float feature groups{tuned}; output {output}")
        unit = f"rank 0's {shard.rows} rows ({shard.nnz} nnz)"
    out = torch.empty((n, F), device=dev) if output == "replicated" else None

    def step():
        if tp is not None:
            return tp.propagate(X0, K, output="sharded")
        return prop.propagate(X0, K, out=out, output=output)
    return step, par, unit


def self_launch(args):
    """`bench.py --gpus N` without torchrun's environment: run
    `python -m torch.distributed.run --nproc-per-node N bench.py <same args>`
    as a child (stdout passes through: rank 0 prints the JSON line) and
    return its exit status (non-zero if any rank failed).  Only
    torch.cuda.device_count() is asked first, which does not initialise the
    runtime."""
    import socket
    import subprocess
    n_dev = torch.cuda.device_count()
    if args.dist_backend == "nccl" and n_dev < args.gpus:
        print(f"bench.py: --gpus {args.gpus} over RCCL needs {args.gpus} GPUs, {n_dev} visible "
              f"(--dist-backend gloo rehearses N ranks sharing the GPUs)", file=sys.stderr)
        return 2
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL on this host
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--shape", default="reddit", choices=sorted(graphs.SHAPES))
    ap.add_argument("--hops", type=int, default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-classifier", action="store_true",
                    help="N=1: skip the classifier sub-record (forward / backward / closure / LBFGS)")
    ap.add_argument("--shapes", default="cora,pubmed,rmat",
                    help="N=1: other BASELINE configs measured into the same line "
                         "(comma list, or 'none')")
    ap.add_argument("--threshold", type=int, default=None, help="heavy-row threshold")
    ap.add_argument("--hub-threshold", type=int, default=None, help="hub-row threshold")
    ap.add_argument("--group-floats", default="auto",
                    help="N>1 rows: feature-group width of the compute/all-gather pipeline "
                         "(an integer, 0 = one full-width group, or auto = timed on this node "
                         "among 0/256/128)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo = host-staged rehearsal of the N>1 path (ranks may share a GPU)")
    ap.add_argument("--distributed-path", action="store_true",
                    help="run the N>1 path even at N=1 (exercises RCCL on one GPU)")
    ap.add_argument("--partition", default="auto",
                    choices=["auto", "rows", "tiles", "cyclic", "features", "lines"],
                    help="N>1: split the rows of S (per-hop all-gather), rows x feature blocks "
                         "(tiles, --col-blocks), round-robin row tiles with column-ordered "
                         "exchange (cyclic), the feature columns (no exchange between hops, "
                         "one all-to-all at the end), or auto = all of them timed on the node")
    ap.add_argument("--cyclic-groups", type=int, default=0,
                    help="N>1 cyclic: column groups (= all-gathers) per hop; 0 = by rank count "
                         "(1 up to 2 ranks, 2 up to 4, else 3: the best of the one-GPU rehearsal, "
                         "DESIGN.md 6.2b)")
    ap.add_argument("--cyclic-tile", type=int, default=64,
                    help="N>1 cyclic: rows per round-robin tile")
    ap.add_argument("--col-blocks", type=int, default=2,
                    help="N>1 tiles: feature blocks C (P = R x C)")
    ap.add_argument("--exchange", default="auto", choices=["auto", "alltoall", "pairwise"],
                    help="feature partition, sharded output: all-to-all after the last hop, or "
                         "pairwise P2P overlapped with it (auto: pairwise at N = 2)")
    ap.add_argument("--chunks", type=int, default=4,
                    help="N>1 features, replicated output: row chunks of the last hop")
    ap.add_argument("--sharded-steps", type=int, default=5,
                    help="N>1: steps timed beside the public call with the partitioned "
                         "propagator and sharded output (0 = skip)")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="schedule knob for sgc_set_tuning (results never depend on it)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: start the ranks here, before anything touches
        # the GPU (no exec after runtime init), relay rank 0's line, and fail
        # if any rank fails
        sys.exit(self_launch(args))
    if args.tune:
        from sgc_amd import _lib
        for kv in args.tune:
            k, v = kv.split("=", 1)
            _lib.check(_lib.load().sgc_set_tuning(k.encode(), int(v)), f"set_tuning {kv}")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    local_dev = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    distributed = world > 1 or args.distributed_path
    if distributed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29555")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)  # RCCL over xGMI
        else:
            dist.init_process_group("gloo")

    spec = graphs.SHAPES[args.shape]
    K = args.hops or spec["hops"]
    lib_sha = lib_sha256()
    metric = (BASELINE_METRIC if args.shape == "reddit" and K == 2 else
              f"propagated edges/sec (K-hop SpMM), {args.shape}-shape K={K}")
    rec = {"metric": metric, "unit": "edges/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "higher_is_better": True, "scaling": "strong",
           "vs_baseline": None, "dtype": "f32",
           "data": "synthetic (seeded R-MAT graph + AugNorm, SURVEY.md 8(d))"}
    if args.tune:
        rec["tuning"] = args.tune

    if not distributed:
        main_rec, S, X_host = single_gpu_shape(args.shape, args, dev, lib_sha, args.steps,
                                               args.warmup, K=K)
        cfg = main_rec.pop("config")
        cfg.update({"parallelism": "single-gpu", "heavy_threshold": args.threshold,
                    "hub_threshold": args.hub_threshold})
        rec.update({"value": main_rec.pop("value"), "ms_per_step": main_rec.pop("ms_per_step"),
                    "config": cfg})
        main_rec.pop("steps"), main_rec.pop("warmup"), main_rec.pop("unit")
        rec.update(main_rec)
        rec["precompute_seconds"] = rec["ms_per_step"] / 1e3
        rec["lib_sha256"] = lib_sha
        if not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(S, X_host)
        del S, X_host
        if not args.no_classifier:
            # the classifier after the precompute (models.py:7-18) and the
            # reference's training closure (reddit.py:51-64) at Reddit-train
            # shape: MFMA forward, weight backward, closure, LBFGS
            from sgc_amd.classifier_bench import classifier_record
            rec["classifier"] = classifier_record(dev)
        subs = [s for s in args.shapes.split(",") if s and s != "none" and s != args.shape]
        if subs:
            rec["shapes"] = {}
            for sh in subs:
                st, wu = SUB_STEPS[sh]
                r, _, _ = single_gpu_shape(sh, args, dev, lib_sha, st, wu)
                r.pop("ms_per_step_events", None)
                rec["shapes"][sh] = r
        print(json.dumps(rec), flush=True)
        return

    S = graphs.synthetic_graph(args.shape, seed=args.seed)
    X_host = graphs.synthetic_features(args.shape, S.n, spec["features"], seed=args.seed + 1)
    n, F, nnz = S.n, X_host.shape[1], S.nnz
    X0 = torch.from_numpy(X_host).to(dev)
    # value: the SAME call as N = 1 -- the reference's sgc_precompute(features,
    # adj, K), unchanged, on every rank under this process group
    # (sgc_amd.utils -> sgc_amd.multigpu: partitioned hops, every rank gets
    # the whole X_K as the reference returns it)
    from sgc_amd import multigpu
    from sgc_amd.distributed import feature_bounds
    from sgc_amd.propagate import warmup
    from sgc_amd.utils import sgc_precompute
    rows_, cols_, vals_ = S.coo()
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.stack([rows_, cols_])),
                                  torch.from_numpy(vals_), (n, n)).to(dev)
    del rows_, cols_, vals_
    torch.cuda.synchronize()
    warm_s = warmup(dev)  # what the drop-in loaders do on every rank
    _, first_pub = sgc_precompute(X0, adj, K)  # ingest + partition set-up + K hops
    partition = multigpu.partition_name(world)
    launches = LaunchTimer(1)

    last = [None]

    def public_step():
        last[0] = sgc_precompute(X0, adj, K)[0]
    elapsed, _, _ = timed(public_step, args.steps, args.warmup, True, dev, events=False)
    # every rank's X_K of the last timed call against the reference's hash
    check = output_check(args.shape, K, last[0], args.seed)
    last[0] = None
    okv = torch.tensor([-1 if check["output_sha_ok"] is None else int(check["output_sha_ok"])],
                       dtype=torch.int32, device=dev if args.dist_backend == "nccl" else "cpu")
    dist.all_reduce(okv, op=dist.ReduceOp.MIN)
    check["output_sha_ok_all_ranks"] = None if int(okv.item()) < 0 else bool(okv.item())
    # the same steps again with the library's per-launch events (rank 0's
    # launches: the roofline's kernel and times; label from the library)
    elapsed_i, step_ms, extra = timed(public_step, args.steps, 1, True, dev,
                                      on_start=launches.start if rank == 0 else None,
                                      on_stop=launches.stop if rank == 0 else None)
    span, light, hub, kernel = extra if extra else (None, None, None, None)
    auto_rec = multigpu.auto_choice(adj._sgc_amd_csr[1], dist.group.WORLD, F, K)
    if partition == "auto" and auto_rec is not None:
        partition = auto_rec["chosen"]
    sharded = None
    if args.sharded_steps > 0:
        # beside it: the partitioned propagator with SHARDED output (each rank
        # keeps its row block of X_K, as a data-parallel classifier would
        # consume it), partition timed on the node (--partition auto)
        tm = {"on": False, "pairs": [], "bytes": []}
        if args.partition == "auto":
            import copy
            cands = ["rows", "cyclic", "features", "lines"]
            if world >= 4 and world % args.col_blocks == 0:
                cands.append("tiles")
            trials = {}
            for cand in cands:
                a = copy.copy(args)
                a.partition = cand
                built = build_dist_step(a, S, X0, dev, rank, world, K, "sharded",
                                        {"on": False, "pairs": [], "bytes": []})
                e_c, _, _ = timed(built[0], 2, 1, True, dev)
                trials[cand] = (e_c / 2, built)
            chosen = min(trials, key=lambda c: (trials[c][0], c))
            step, par, _ = trials[chosen][1]
            par += " [auto-selected: " + ", ".join(f"{c} {trials[c][0] * 1e3:.2f} ms"
                                                   for c in cands) + "]"
        else:
            step, par, _ = build_dist_step(args, S, X0, dev, rank, world, K, "sharded", tm)
        e_sh, _, _ = timed(step, args.sharded_steps, 1, True, dev)
        sharded = {"output": "sharded (each rank: its row block of X_K)", "parallelism": par,
                   "steps": args.sharded_steps, "ms_per_step": e_sh * 1e3 / args.sharded_steps,
                   "value": K * nnz * args.sharded_steps / e_sh,
                   "what": "the partitioned propagator without the final replication; not the "
                           "reference's call"}
    if rank == 0:
        fb, B = feature_bounds(F, world)
        par = (f"{partition}-partition x{world} via sgc_precompute under the process group "
               f"({'RCCL over xGMI' if args.dist_backend == 'nccl' else 'gloo rehearsal'}); "
               f"output replicated (every rank gets all of X_K, as the reference returns it)")
        rec.update({"value": K * nnz * args.steps / elapsed,
                    "ms_per_step": elapsed * 1e3 / args.steps,
                    "ms_per_step_median_rank0": float(np.median(step_ms)),
                    "ms_per_step_instrumented": elapsed_i * 1e3 / args.steps,
                    "config": {"workload": f"{args.shape}-shape sgc_precompute K={K}", "nodes": n,
                               "undirected_edges": spec["edges"], "nnz": nnz, "features": F,
                               "hops": K, "parallelism": par, "output": "replicated",
                               "partition": partition,
                               "auto_seconds": None if auto_rec is None else auto_rec["seconds"]},
                    "timed_call": "sgc_precompute(features, adj, K) (sgc_amd.utils, the drop-in), "
                                  "every rank, the same call as N = 1",
                    "first_call_seconds": round(first_pub, 4),
                    "loader_warmup_seconds": round(warm_s, 4),
                    "lib_sha256": lib_sha})
        rec.update(check)
        if span:
            # rank 0's SpMM launches over one step: the compulsory bytes of its
            # K hops (S once, its block of X once, its Y once -- the same model
            # as N = 1's `compulsory_frac`) over the launches' summed spans
            # (launches on concurrent streams counted in full: conservative)
            cb = None
            if partition == "replicate":
                cb = K * (4 * (n + 1) + 8 * nnz + 8 * F * n)
                unit = f"rank 0's K hops over all {n} rows at all {F} columns (replicate)"
            elif partition == "features":
                w = int(fb[1] - fb[0])
                cb = K * (4 * (n + 1) + 8 * nnz + 8 * w * n)
                unit = f"rank 0's K hops over all {n} rows at its {w}-column block"
            elif partition == "lines":
                from sgc_amd.distributed import line_bounds, nnz_balanced_bounds
                W, T = line_bounds(F, world)
                wt = F - T
                b = nnz_balanced_bounds(S.row_ptr, world)
                rows0 = int(b[1] - b[0])
                nnz0 = int(S.row_ptr[b[1]] - S.row_ptr[b[0]])
                cb = K * ((4 * (n + 1) + 8 * nnz + 8 * min(W, F) * n if W else 0) +
                          (4 * (rows0 + 1) + 8 * nnz0 + 4 * wt * (n + rows0) if wt else 0))
                unit = (f"rank 0's K hops: all {n} rows at its {W}-column line block + its "
                        f"{rows0} tail rows at the {wt} tail columns")
            t_step = float(np.sum(span)) * 1e-3 / args.steps
            rec["roofline"] = {
                "bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "kernel": (f"{kernel} (+ spmm_hub_kernel beside it, joined)" if hub else
                           str(kernel)),
                "kernel_mean_ms": float(np.mean(span)), "launches": len(span),
                "launch_unit": unit if cb else "rank 0's SpMM launches",
                "launch_ms_per_step": t_step * 1e3,
                "achieved": cb / t_step / 1e9 if cb else None,
                "frac": cb / t_step / 1e9 / HBM_PEAK_GBS if cb else None,
                "compulsory_bytes_per_step": cb,
                "compulsory_frac": cb / t_step / 1e9 / HBM_PEAK_GBS if cb else None,
                "traffic": None,
                "achieved_basis": "compulsory bytes (S, the block of X and its Y once) of rank "
                                  "0's launches per step over their summed spans; N = 1's "
                                  "roofline carries the same basis as compulsory_frac"}
        rec["precompute_seconds"] = rec["ms_per_step"] / 1e3
        if sharded is not None:
            rec["sharded_output"] = sharded
        print(json.dumps(rec), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
