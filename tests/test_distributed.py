"""Row-partitioned propagation (sgc_amd.distributed) over gloo, world_size 2-4, CPU.

The exchange logic (nnz-balanced bounds, padded column remap, per-hop
all_gather_into_tensor, final compaction) is exercised with the CPU oracle
injected as the per-rank SpMM; the result must equal the single-process
golden output bit for bit.  The GPU runs the same class with the HIP kernel
and RCCL (bench.py --gpus N).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from sgc_amd.distributed import (RowPartitionedPropagator, equal_row_bounds, make_shard,
                                 nnz_balanced_bounds)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bounds_balance_nnz():
    rp = np.array([0, 100, 101, 102, 103, 203, 204, 205, 305])
    b = nnz_balanced_bounds(rp, 3)
    assert b[0] == 0 and b[-1] == 8 and np.all(np.diff(b) >= 0)
    loads = [rp[b[i + 1]] - rp[b[i]] for i in range(3)]
    assert max(loads) <= 2 * rp[-1] / 3
    # more ranks than rows -> empty shards are fine
    b = nnz_balanced_bounds(np.array([0, 5, 10]), 4)
    assert b[0] == 0 and b[-1] == 2 and np.all(np.diff(b) >= 0)


def test_equal_row_bounds():
    assert equal_row_bounds(10, 4).tolist() == [0, 3, 6, 9, 10]
    assert equal_row_bounds(2, 4).tolist() == [0, 1, 2, 2, 2]
    assert equal_row_bounds(8, 2).tolist() == [0, 4, 8]


def _oracle_spmm(shard, X, out):
    from oracle import oracle as o
    rp = shard.row_ptr.numpy()
    Y = o.spmm_csr(rp, shard.col_idx.numpy(), shard.val.numpy(), X.numpy())
    out.copy_(torch.from_numpy(Y))
    return out


def _worker(rank, world, port, case, K, result_q, group_floats=128, staging=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as o
        n = int(case["n"])
        rp, ci, va = o.coo_to_csr(n, n, case["rows"], case["cols"], case["vals"])
        shard = make_shard(rp, ci, va, rank, world, "cpu")
        prop = RowPartitionedPropagator(shard, spmm_fn=_oracle_spmm, group_floats=group_floats,
                                        host_staging=staging)
        X0 = torch.from_numpy(case["X"])
        out = prop.propagate(X0, K)
        result_q.put((rank, out.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,name,K,gf,staging", [
    (2, "norm_n48_F65", 2, 128, False), (2, "hub1000_F65", 2, 16, False),
    (3, "norm_n48_F602", 3, 128, False), (4, "raw_unsorted_dups_F7", 3, 2, False),
    (2, "isolated_F17", 1, 4, True), (2, "norm_n48_F130", 2, 64, True)])
def test_row_partition_gloo_bit_exact(tiny_cases, oracle, world, name, K, gf, staging):
    case = tiny_cases[name]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, K, q, gf, staging))
             for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = case[f"Y{K}"]
    for r in range(world):
        assert np.array_equal(results[r].view(np.uint32), want.view(np.uint32)), (name, r)
