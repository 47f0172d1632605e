"""bench.py -- SGC propagation hot path on MI355X: propagated edges/s.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--shape reddit]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Metric (BASELINE.json): propagated edges/s = hops * nnz(S) / t, where t is
one sgc_precompute (all K hops of S.X, reference utils.py:92-97) over the
synthetic Reddit-shape graph (232,965 nodes, 11,606,919 undirected edges,
nnz(S) = 23,446,803, F = 602, K = 2), inputs resident in HBM.
A "step" = one full K-hop propagation.  N > 1 (sgc_amd.distributed), total
work fixed, so scaling is "strong":
  --partition rows (default)  S row-partitioned (equal-row blocks, SURVEY.md
                8(e)); RCCL all-gather of X_k after each hop that feeds another,
                pipelined in 128-float feature groups
  --partition features  each rank runs all K hops on its block of feature
                columns over the full S, no exchange between hops
  --output sharded (default)  each rank ends with its row block of X_K -- the
                layout the data-parallel classifier consumes
                (sgc_amd.distributed.ShardedSGCTrainer); no gather after the
                last hop (rows) / one all-to-all (features)
  --output replicated  every rank ends with all of X_K (one more all-gather)
The other output mode is timed too (`alt_output`, --alt-steps).

Also printed (same JSON line):
  roofline      dominant kernel (the CSR SpMM) -- algorithmic bytes per hop
                (gather model: 4(N+1) + 8nnz + 4F nnz + 4F N) / the kernel's
                mean duration measured with events on the launch stream;
                `traffic` = HBM bytes per launch from rocprofv3 PMC counters
                when profiles/pmc_<shape>.json exists (else null)
  cpu_baseline  the reference's arithmetic as written -- torch.spmm(COO, X)
                (utils.py:95) on this host's CPU, one hop, rank 0 at N = 1
"""
import argparse
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
from sgc_amd.propagate import DeviceCSR, propagate  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
BASELINE_METRIC = ("propagated edges/sec (K-hop SpMM) + precompute wall-time, "
                   "Reddit K=2 at 1/2/4/8 GPUs")


def algorithmic_bytes_per_hop(n, nnz, F):
    return 4 * (n + 1) + 8 * nnz + 4 * F * nnz + 4 * F * n


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def cpu_baseline(S, X_host, budget_s=30.0):
    """The reference's arithmetic on this host: torch.spmm(COO, X) -- what
    utils.py:95 runs each hop.  One hop over the full graph after a warm-up
    hop on 64 feature columns (allocator first touch).  aten's COO kernel is
    single-threaded whatever torch.get_num_threads() says, so
    cores = 1.  Also times the CSR variant at all threads (bit-identical
    output, the best CPU torch path) when the budget allows."""
    rows, cols, vals = S.coo()
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.stack([rows, cols])),
                                  torch.from_numpy(vals), (S.n, S.n))
    X = torch.from_numpy(X_host)
    torch.spmm(adj, X[:, :64].contiguous())
    t0 = time.perf_counter()
    torch.spmm(adj, X)
    t_coo = time.perf_counter() - t0
    rec = {"value": S.nnz / t_coo, "unit": "edges/s", "cores": 1, "kind": "reference",
           "sample": f"1 hop of torch.spmm(COO fp32 {S.n}x{S.n}, nnz {S.nnz}; X [{S.n},{X.shape[1]}]) "
                     f"on the host CPU = reference utils.py:95 as written, after a 64-column "
                     f"warm-up; {t_coo:.2f} s",
           "host_cpu": cpu_model(), "os_cpu_count": os.cpu_count(),
           "torch_threads": torch.get_num_threads()}
    if t_coo < budget_s / 3:
        csr = adj.to_sparse_csr()
        torch.sparse.mm(csr, X)
        t0 = time.perf_counter()
        torch.sparse.mm(csr, X)
        t_csr = time.perf_counter() - t0
        rec["csr_all_threads"] = {"value": S.nnz / t_csr, "unit": "edges/s",
                                  "cores": torch.get_num_threads(), "seconds": round(t_csr, 3)}
    return rec


def load_traffic(shape):
    p = os.path.join(ROOT, "profiles", f"pmc_{shape}.json")
    if not os.path.exists(p):
        return None, None
    with open(p) as f:
        d = json.load(f)
    return d.get("hbm_bytes_per_launch"), os.path.relpath(p, ROOT)


def build_step(args, S, X0, dev, rank, world, distributed, K, output, timing):
    """(step, parallelism, launch description) for one output mode.  timing =
    {"on", "starts", "ends", "bytes"}: every SpMM launch is bracketed by HIP
    events on its stream while timing["on"]."""
    n, F = X0.shape

    def bracket(fn, nbytes):
        def run(*a, **k):
            if not timing["on"]:
                return fn(*a, **k)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            r = fn(*a, **k)
            e.record()
            timing["starts"].append(s)
            timing["ends"].append(e)
            timing["bytes"].append(nbytes(*a))
            return r
        return run

    if not distributed:
        csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device=dev)
        csr.plan(0, n, args.threshold, args.hub_threshold, F)
        out_buf = torch.empty((n, F), device=dev)
        ev = {}

        def hook(phase, h):
            if not timing["on"]:
                return
            if phase == "start":
                ev["s"] = torch.cuda.Event(enable_timing=True)
                ev["s"].record()
            else:
                e = torch.cuda.Event(enable_timing=True)
                e.record()
                timing["starts"].append(ev["s"])
                timing["ends"].append(e)
                timing["bytes"].append(algorithmic_bytes_per_hop(n, S.nnz, F))

        def step():  # the product path of sgc_precompute (sgc_amd.propagate)
            return propagate(csr, X0, K, out=out_buf, threshold=args.threshold, hop_hook=hook,
                             hub_threshold=args.hub_threshold)
        return step, "single-gpu", f"one hop over all {n} rows"

    backend = "rccl" if args.dist_backend == "nccl" else "gloo rehearsal"
    staging = args.dist_backend == "gloo"
    if args.partition == "features":
        from sgc_amd.distributed import FeaturePartitionedPropagator, feature_bounds
        from sgc_amd.propagate import spmm as spmm_hip
        csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device=dev)
        rp = np.asarray(S.row_ptr, dtype=np.int64)

        def launch_bytes(X, r0, r1, out):
            nz, w = int(rp[r1] - rp[r0]), X.shape[1]
            return 4 * (r1 - r0 + 1) + 8 * nz + 4 * w * nz + 4 * w * (r1 - r0)

        spmm_fn = bracket(lambda X, r0, r1, out: spmm_hip(
            csr, X, r0, r1, out=out, threshold=args.threshold,
            hub_threshold=args.hub_threshold), launch_bytes)
        prop = FeaturePartitionedPropagator(csr, rank=rank, world_size=world, spmm_fn=spmm_fn,
                                            chunks=args.chunks, host_staging=staging)
        fb, fB = feature_bounds(F, world)
        exch = ("one all-to-all of the row blocks of X_K" if output == "sharded" else
                f"one all-gather of X_K pipelined with the last hop in {args.chunks} row chunks")
        par = (f"feature-partition x{world} ({fB}-column blocks, all K hops local) + {backend} "
               f"{exch}; output {output}")
        unit = (f"rank 0's SpMM launches (mean): hops over all {n} rows or last-hop row blocks, "
                f"{int(fb[1] - fb[0])} feature columns")
    else:
        from sgc_amd.distributed import RowPartitionedPropagator, _default_spmm, make_shard
        shard = make_shard(S.row_ptr, S.col_idx, S.val, rank, world, dev)
        nnz_l = shard.nnz

        def launch_bytes(sh, X, out):
            fg = X.shape[1]
            return 4 * (sh.rows + 1) + 8 * nnz_l + 4 * fg * nnz_l + 4 * fg * sh.rows

        auto = args.group_floats == "auto"
        prop = RowPartitionedPropagator(shard, spmm_fn=bracket(_default_spmm, launch_bytes),
                                        group_floats=224 if auto else int(args.group_floats),
                                        host_staging=staging)
        tuned = ""
        if auto:  # untimed setup, like the plans: every rank picks the same width
            tt = prop.autotune(X0, K, output=output)
            tuned = " (autotuned: " + ", ".join(f"{g}: {t * 1e3:.2f} ms"
                                                for g, t in tt.items()) + ")"
        gf = prop.group_floats
        exch = ("all-gather of X_k after each hop but the last" if output == "sharded" else
                "all-gather of X_k after every hop")
        par = (f"row-partition x{world} (equal-row blocks) + {backend} {exch}, pipelined in "
               f"{gf}-float feature groups{tuned}; output {output}")
        unit = (f"one hop of one {gf}-float feature group over rank 0's "
                f"{shard.rows} rows ({nnz_l} nnz)")
    out = None
    if output == "replicated":
        out = torch.empty((n, F), device=dev)

    def step():
        return prop.propagate(X0, K, out=out, output=output)
    return step, par, unit


def timed(step, steps, warmup, distributed, dev, timing):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    timing["on"] = True
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    timing["on"] = False
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    return elapsed


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--shape", default="reddit", choices=sorted(graphs.SHAPES))
    ap.add_argument("--hops", type=int, default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--threshold", type=int, default=None, help="heavy-row threshold")
    ap.add_argument("--hub-threshold", type=int, default=None, help="hub-row threshold")
    ap.add_argument("--group-floats", default="auto",
                    help="N>1 rows: feature-group width of the compute/all-gather pipeline "
                         "(an integer, or auto = timed on this node among 224/304/160)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo = host-staged rehearsal of the N>1 path (ranks may share a GPU)")
    ap.add_argument("--distributed-path", action="store_true",
                    help="run the N>1 path even at N=1 (exercises RCCL on one GPU)")
    ap.add_argument("--partition", default="rows", choices=["rows", "features"],
                    help="N>1: split the rows of S (per-hop all-gather) or the feature columns")
    ap.add_argument("--output", default="sharded", choices=["sharded", "replicated"],
                    help="N>1: each rank keeps its row block of X_K, or all ranks get all of it")
    ap.add_argument("--chunks", type=int, default=4,
                    help="N>1 features, replicated output: row chunks of the last hop")
    ap.add_argument("--alt-steps", type=int, default=5,
                    help="N>1: steps timed with the other output mode (0 = skip)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N>1 must be launched with torch.distributed.run")
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
    t_gen = time.perf_counter()
    S = graphs.synthetic_graph(args.shape, seed=args.seed)
    X_host = graphs.synthetic_features(args.shape, S.n, spec["features"], seed=args.seed + 1)
    t_gen = time.perf_counter() - t_gen
    n, F, nnz = S.n, X_host.shape[1], S.nnz
    X0 = torch.from_numpy(X_host).to(dev)

    timing = {"on": False, "starts": [], "ends": [], "bytes": []}
    step, parallelism, unit_desc = build_step(args, S, X0, dev, rank, world, distributed, K,
                                              args.output, timing)
    elapsed = timed(step, args.steps, args.warmup, distributed, dev, timing)
    kern_ms = [s.elapsed_time(e) for s, e in zip(timing["starts"], timing["ends"])]
    bytes_launch = float(np.mean(timing["bytes"])) if timing["bytes"] else float("nan")

    ms_per_step = elapsed * 1e3 / args.steps
    value = K * nnz * args.steps / elapsed
    kern_mean_ms = float(np.mean(kern_ms)) if kern_ms else float("nan")
    achieved = bytes_launch / (kern_mean_ms * 1e-3) / 1e9
    traffic, traffic_src = load_traffic(args.shape) if not distributed else (None, None)

    alt = None
    if distributed and args.alt_steps > 0:
        alt_mode = "replicated" if args.output == "sharded" else "sharded"
        t_alt = {"on": False, "starts": [], "ends": [], "bytes": []}
        alt_step, alt_par, _ = build_step(args, S, X0, dev, rank, world, distributed, K, alt_mode,
                                          t_alt)
        e_alt = timed(alt_step, args.alt_steps, 1, distributed, dev, t_alt)
        alt = {"output": alt_mode, "parallelism": alt_par, "steps": args.alt_steps,
               "ms_per_step": e_alt * 1e3 / args.alt_steps,
               "value": K * nnz * args.alt_steps / e_alt}

    rec = None
    if rank == 0:
        rec = {
            "metric": (BASELINE_METRIC if args.shape == "reddit" and K == 2 else
                       f"propagated edges/sec (K-hop SpMM), {args.shape}-shape K={K}"),
            "value": value,
            "unit": "edges/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded R-MAT graph + AugNorm, SURVEY.md 8(d))",
            "config": {"workload": f"{args.shape}-shape sgc_precompute K={K}", "nodes": n,
                       "undirected_edges": spec["edges"], "nnz": nnz, "features": F, "hops": K,
                       "parallelism": parallelism, "heavy_threshold": args.threshold,
                       "hub_threshold": args.hub_threshold},
            "precompute_seconds": ms_per_step / 1e3,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "spmm_csr_kernel + spmm_hub_kernel (side stream, joined)",
                         "kernel_mean_ms": kern_mean_ms,
                         "algorithmic_bytes_per_launch": bytes_launch,
                         "launch_unit": unit_desc, "traffic_source": traffic_src,
                         "compulsory_bytes_per_hop": 4 * (n + 1) + 8 * nnz + 8 * F * n},
            "generate_seconds": round(t_gen, 2),
        }
        if alt is not None:
            rec["alt_output"] = alt
        if world == 1 and not distributed and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(S, X_host)
        print(json.dumps(rec), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
