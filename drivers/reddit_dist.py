"""Multi-GPU Reddit driver: the reference reddit.py flow (transductive,
reddit.py:36-74) with the precompute row-partitioned over the GPUs and the
classifier trained data-parallel -- nothing ever holds all of X_K.

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
        drivers/reddit_dist.py [--synthetic 232965] [--test] [--degree 2] [--epochs 2]

Every rank builds the same seeded Reddit-shape graph (sgc_amd.graphs, the
SURVEY.md 8(d) recipe), labels and splits, keeps its equal-row block of S,
and runs:
  precompute  RowPartitionedPropagator(output="sharded"): K hops, an RCCL
              all-gather of X_k between hops, this rank's rows of X_K out;
  train       reddit.py:51-64's LBFGS(lr=1) over ShardedSGCTrainer -- the
              fused loss/gradient kernel on the rank's training rows and one
              all-reduce of [loss, dW, db] per closure;
  test        micro/macro F1 (metrics.py:9-15, sklearn's definitions) from
              per-class true-positive / predicted / actual counts summed over
              the ranks.
Rank 0 prints the reference's line: "Total Time: ...s, Test F1: ...".
--check (world size 1 only) also runs the single-GPU path (sgc_precompute +
SGC + torch LBFGS) and compares: X_K bit for bit; F1 within 0.01 (the
data-parallel gradients differ from torch's in rounding, which LBFGS may
amplify into a few flipped predictions).
"""
import argparse
import os
import sys
from time import perf_counter

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sgc_amd import graphs  # noqa: E402
from sgc_amd.distributed import (RowPartitionedPropagator, ShardedSGCTrainer,  # noqa: E402
                                 make_shard)
from sgc_amd.models import SGC  # noqa: E402

N_CLASSES = 41


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--synthetic", type=int, default=graphs.SHAPES["reddit"]["n"],
                   help="nodes of the seeded Reddit-shape graph")
    p.add_argument("--test", action="store_true")
    p.add_argument("--degree", type=int, default=2)
    p.add_argument("--epochs", type=int, default=2)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--check", action="store_true", help="world size 1: compare with 1-GPU path")
    return p.parse_args(argv)


def dataset(n, seed):
    spec = graphs.SHAPES["reddit"]
    edges = max(1, int(spec["edges"] * n / spec["n"]))
    S = graphs.synthetic_graph("reddit", seed=0, n=n, edges=edges)
    X = graphs.synthetic_features("reddit", S.n, spec["features"], seed=1)
    rng = np.random.default_rng(seed)
    perm = rng.permutation(S.n)
    a, b = int(0.66 * S.n), int(0.76 * S.n)
    splits = {"train": np.sort(perm[:a]), "val": np.sort(perm[a:b]), "test": np.sort(perm[b:])}
    # labels that depend on the graph (so training is not on pure noise):
    # the class of each node's largest feature among the first 41
    labels = np.argmax(X[:, :N_CLASSES], axis=1).astype(np.int64)
    return S, X, labels, splits


def f1_from_counts(tp, pred, true):
    """sklearn f1_score(average='micro'/'macro') from per-class counts."""
    micro = 2 * tp.sum() / max(1, pred.sum() + true.sum())
    denom = pred + true
    per = np.where(denom > 0, 2 * tp / np.maximum(denom, 1), 0.0)
    present = (true > 0) | (pred > 0)  # labels present in y_true or y_pred
    macro = per[present].mean() if present.any() else 0.0
    return float(micro), float(macro)


def main(argv=None):
    args = parse(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    os.environ.setdefault("RANK", str(rank))
    os.environ.setdefault("WORLD_SIZE", str(world))
    dist.init_process_group("nccl", device_id=dev)
    torch.manual_seed(args.seed)

    S, X_host, labels_host, splits = dataset(args.synthetic, args.seed)
    X0 = torch.from_numpy(X_host).to(dev)
    labels = torch.from_numpy(labels_host).to(dev)
    shard = make_shard(S.row_ptr, S.col_idx, S.val, rank, world, dev)
    r0, r1 = shard.row_begin, shard.row_end
    if rank == 0:
        print("Finished data loading.", flush=True)

    model = SGC(X_host.shape[1], N_CLASSES).to(dev)
    for p in model.parameters():  # one initialisation for all ranks
        dist.broadcast(p.data, src=0)

    prop = RowPartitionedPropagator(shard)
    torch.cuda.synchronize()
    dist.barrier()
    t = perf_counter()
    X_rows = prop.propagate(X0, args.degree, output="sharded")  # rows [r0, r1) of X_K
    torch.cuda.synchronize()
    dist.barrier()
    precompute_time = perf_counter() - t

    def local_split(name):
        idx = splits[name]
        idx = idx[(idx >= r0) & (idx < r1)]
        sel = torch.from_numpy(idx - r0).to(dev)
        return X_rows.index_select(0, sel), labels[torch.from_numpy(idx).to(dev)]

    Xtr, ytr = local_split("train")
    trainer = ShardedSGCTrainer(model)
    opt = torch.optim.LBFGS(model.parameters(), lr=1)
    m_train = len(splits["train"])

    def closure():
        opt.zero_grad()
        return trainer.loss(Xtr, ytr, m_train)

    t = perf_counter()
    for _ in range(args.epochs):
        opt.step(closure)
    torch.cuda.synchronize()
    train_time = perf_counter() - t

    Xte, yte = local_split("test" if args.test else "val")
    with torch.no_grad():
        pred = model(Xte).argmax(dim=1) if Xte.shape[0] else yte
    counts = torch.zeros((3, N_CLASSES), dtype=torch.float64, device=dev)
    if Xte.shape[0]:
        ones = torch.ones_like(pred, dtype=torch.float64)
        counts[0].index_add_(0, pred[pred == yte], ones[pred == yte])
        counts[1].index_add_(0, pred, ones)
        counts[2].index_add_(0, yte, ones)
    dist.all_reduce(counts)
    micro, macro = f1_from_counts(*counts.cpu().numpy())
    if rank == 0:
        print("Total Time: {:.4f}s, {} F1: {:.4f}".format(train_time + precompute_time,
                                                          "Test" if args.test else "Val", micro),
              flush=True)
        print(f"precompute {precompute_time * 1e3:.2f} ms over {world} GPU(s), "
              f"train {train_time * 1e3:.2f} ms, macro F1 {macro:.4f}", flush=True)

    if args.check and world == 1:
        check(args, S, X0, labels, splits, X_rows, micro, dev)
    dist.barrier()
    dist.destroy_process_group()
    return micro


def check(args, S, X0, labels, splits, X_rows, micro, dev):
    """1-GPU reference path on the same inputs: reddit.py as written."""
    import torch.nn.functional as F

    from sgc_amd.metrics import f1
    from sgc_amd.propagate import DeviceCSR, propagate
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device=dev)
    full = propagate(csr, X0, args.degree)
    assert torch.equal(full, X_rows), "sharded X_K differs from the 1-GPU X_K"
    torch.manual_seed(args.seed)
    model = SGC(X0.shape[1], N_CLASSES).to(dev)
    opt = torch.optim.LBFGS(model.parameters(), lr=1)
    tr = torch.from_numpy(splits["train"]).to(dev)

    def closure():
        opt.zero_grad()
        loss = F.cross_entropy(model(full[tr]), labels[tr])
        loss.backward()
        return loss
    for _ in range(args.epochs):
        opt.step(closure)
    te = torch.from_numpy(splits["test" if args.test else "val"]).to(dev)
    ref_micro, _ = f1(model(full[te]), labels[te])
    print(f"check: X_K bit-identical; F1 {micro:.6f} vs 1-GPU {ref_micro:.6f}", flush=True)
    assert abs(micro - ref_micro) <= 0.01, (micro, ref_micro)


if __name__ == "__main__":
    main()
