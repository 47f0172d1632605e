"""Bit-exactness of the N-rank paths at full BASELINE size, rehearsed on ONE GPU.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        scripts/dist_check.py [--shape reddit] [--partition rows|tiles|cyclic|features|lines]
                              [--col-blocks 2]

Every rank drives the same GPU (cuda:0) with the gloo backend (host-staged
all-gathers, so no RCCL peer access is needed), runs the exact product
propagator of bench.py (nnz-balanced row blocks, split hub launches, the
autotuned pipeline) and keeps its sharded rows of X_K; rank 0 collects every
block and compares the SHA-256 of the assembled X_K with the reference's own
golden (tests/golden/shapes.json).  One JSON line from rank 0.
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from sgc_amd import graphs  # noqa: E402
from sgc_amd.distributed import RowPartitionedPropagator, TiledPropagator, make_shard  # noqa: E402


def _sha(t):
    return hashlib.sha256(t.cpu().numpy().tobytes()).hexdigest()


def replicated_checks(prop, X, K, g):
    """The replicated output on this rank -- every rank's full X_K -- through
    the default exchange on the GPU (IPC pulls of the peers' blocks, no
    gathered copy) and through the collective one (in-place all-gathers +
    unpack): both against the reference's hash.  Then three IPC calls with
    X, 2X and 4X: S^K (2^j X) = 2^j S^K X bit for bit (power-of-two scaling
    is exact through every fma), and the calls alternate the window's two
    halves, so a block left over from an earlier call would show."""
    want = g["outputs"][str(K)]["sha"]
    os.environ["SGC_AMD_REPLICATED_EXCHANGE"] = "collective"
    coll = prop.propagate(X, K, output="replicated")
    rec = {"collective_sha_ok": _sha(coll) == want}
    del coll
    os.environ.pop("SGC_AMD_REPLICATED_EXCHANGE")
    outs = [prop.propagate(X * float(2 ** j), K, output="replicated") for j in range(3)]
    torch.cuda.synchronize()
    rec["default_sha_ok"] = _sha(outs[0]) == want
    rec["scaled_calls_exact"] = all(torch.equal(outs[j], outs[0] * float(2 ** j)) for j in (1, 2))
    rec["exchange"] = "ipc" if getattr(prop, "_ipc", None) is not None else "collective"
    rec["ipc_unavailable"] = getattr(prop, "ipc_unavailable", None) or ""
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="reddit")
    ap.add_argument("--partition", default="rows", choices=["rows", "tiles", "cyclic", "features", "lines"])
    ap.add_argument("--groups", type=int, default=4, help="cyclic: column groups")
    ap.add_argument("--tile", type=int, default=64, help="cyclic: rows per tile")
    ap.add_argument("--col-blocks", type=int, default=2)
    ap.add_argument("--row-chunks", type=int, default=1)
    ap.add_argument("--group-floats", type=int, default=0)
    ap.add_argument("--exchange", default="auto", choices=["auto", "alltoall", "pairwise"],
                    help="features: the sharded exchange")
    ap.add_argument("--pieces", type=int, default=None, help="features: pairwise row pieces")
    ap.add_argument("--also-replicated", action="store_true",
                    help="lines / features: also check the replicated output (IPC and "
                         "collective exchanges) against the reference hash")
    ap.add_argument("--device", default="cuda", help="cpu: the CPU-twin rehearsal")
    ap.add_argument("--cache", default=os.environ.get("TMPDIR", "/tmp"))
    args = ap.parse_args()
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    if args.device == "cuda":
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
    else:
        dev = torch.device("cpu")
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "shapes.json")))[args.shape]
    spec = graphs.SHAPES[args.shape]
    t0 = time.time()
    # rank 0 generates the inputs once and shares them through .npy files
    # (the RMAT shape takes minutes to generate; eight copies would thrash)
    cache = os.path.join(args.cache, f"dist_check_{args.shape}")
    names = ("row_ptr", "col_idx", "val", "X")
    cached = all(os.path.exists(os.path.join(cache, nm + ".npy")) for nm in names)
    if rank == 0 and not cached:
        S = graphs.synthetic_graph(args.shape, seed=g["seed"])
        Xh = graphs.synthetic_features(args.shape, g["n"], g["features"], seed=g["feature_seed"])
        if world > 1:
            os.makedirs(cache, exist_ok=True)
            for name, arr in zip(names, (S.row_ptr, S.col_idx, S.val, Xh)):
                np.save(os.path.join(cache, name + ".npy"), arr)
    dist.barrier()
    if rank != 0 or cached:
        ld = lambda name: np.load(os.path.join(cache, name + ".npy"), mmap_mode="r")  # noqa: E731
        S = graphs.CSRGraph(g["n"], ld("row_ptr"), ld("col_idx"), ld("val"))
        Xh = ld("X")
    X = torch.from_numpy(np.ascontiguousarray(Xh)).to(dev)
    del Xh
    K = spec["hops"]
    row_index = None
    replicated = None
    if args.partition == "cyclic":
        from sgc_amd.distributed import CyclicRowPropagator
        cp = CyclicRowPropagator(S.row_ptr, S.col_idx, S.val, rank, world, dev, tile=args.tile,
                                 groups=args.groups, host_staging=True)
        mine = cp.propagate(X, K, output="sharded")
        row_index = cp.row_index
        r0, r1 = 0, 0
    elif args.partition == "features":
        from sgc_amd.distributed import FeaturePartitionedPropagator, equal_row_bounds
        from sgc_amd.propagate import DeviceCSR
        csr = DeviceCSR.from_host_arrays(np.asarray(S.row_ptr), np.asarray(S.col_idx),
                                         np.asarray(S.val), device=dev)
        fp = FeaturePartitionedPropagator(csr, host_staging=True, exchange=args.exchange,
                                          pieces=args.pieces)
        mine = fp.propagate(X, K, output="sharded")
        if args.also_replicated:
            replicated = replicated_checks(fp, X, K, g)
        rb = equal_row_bounds(g["n"], world)
        r0, r1 = int(rb[rank]), int(rb[rank + 1])
    elif args.partition == "lines":
        from sgc_amd.distributed import LinePartitionedPropagator, equal_row_bounds
        from sgc_amd.propagate import DeviceCSR
        csr = DeviceCSR.from_host_arrays(np.asarray(S.row_ptr), np.asarray(S.col_idx),
                                         np.asarray(S.val), device=dev)
        shard = make_shard(S.row_ptr, S.col_idx, S.val, rank, world, dev)
        lp = LinePartitionedPropagator(shard, csr=csr, host_staging=True)
        mine = lp.propagate(X, K, output="sharded")
        if args.also_replicated:  # every rank's full X_K must equal the sharded rows
            replicated = replicated_checks(lp, X, K, g)
            full = lp.propagate(X, K, output="replicated")
            rb = equal_row_bounds(g["n"], world)
            assert torch.equal(full[int(rb[rank]):int(rb[rank + 1])], mine)
        rb = equal_row_bounds(g["n"], world)
        r0, r1 = int(rb[rank]), int(rb[rank + 1])
    elif args.partition == "tiles":
        tp = TiledPropagator(S.row_ptr, S.col_idx, S.val, rank, world, args.col_blocks, dev,
                             group_floats=args.group_floats, host_staging=True)
        tp.prop.row_chunks = args.row_chunks
        mine = tp.propagate(X, K, output="sharded")
        r0, r1 = tp.row_begin, tp.row_end
    else:
        shard = make_shard(S.row_ptr, S.col_idx, S.val, rank, world, dev)
        prop = RowPartitionedPropagator(shard, group_floats=args.group_floats, host_staging=True,
                                        row_chunks=args.row_chunks)
        mine = prop.propagate(X, K, output="sharded")
        r0, r1 = shard.row_begin, shard.row_end
    if dev.type == "cuda":
        torch.cuda.synchronize()
    blocks = [None] * world if rank == 0 else None
    dist.gather_object((r0, r1, row_index, mine.cpu().numpy()), blocks, dst=0)
    reps = [None] * world if rank == 0 else None
    dist.gather_object(replicated, reps, dst=0)
    if rank == 0:
        Y = np.empty((g["n"], g["features"]), np.float32)
        covered = np.zeros(g["n"], bool)
        for a, b, ri, arr in blocks:
            if ri is not None:  # cyclic: the rank's rows by global id
                assert not covered[ri].any()
                Y[ri] = arr
                covered[ri] = True
            elif b > a and not covered[a:b].any():  # tiles: C ranks share a row block
                Y[a:b] = arr
                covered[a:b] = True
        ok = bool(covered.all()) and hashlib.sha256(Y.tobytes()).hexdigest() == \
            g["outputs"][str(K)]["sha"]
        print(json.dumps({"shape": args.shape, "world": world, "partition": args.partition,
                          "col_blocks": args.col_blocks if args.partition == "tiles" else 1,
                          "row_chunks": args.row_chunks, "group_floats": args.group_floats,
                          "groups": args.groups if args.partition == "cyclic" else None,
                          "rows_per_rank": [int(b - a) if ri is None else int(len(ri))
                                            for a, b, ri, _ in blocks],
                          "bit_exact_vs_reference_hash": ok,
                          "replicated": None if replicated is None else {
                              k: all(r[k] for r in reps) for k in replicated
                              if isinstance(replicated[k], bool)},
                          "replicated_exchange": None if replicated is None else
                              sorted({r["exchange"] for r in reps}),
                          "seconds": round(time.time() - t0, 1)}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
