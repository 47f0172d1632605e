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

from sgc_amd.distributed import (FeaturePartitionedPropagator, LinePartitionedPropagator,
                                 RowPartitionedPropagator, equal_row_bounds, feature_bounds,
                                 line_bounds, make_shard, nnz_balanced_bounds, row_chunks)


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


def _oracle_spmm(shard, X, out, layout="input", part="all", rows=None):
    from oracle import oracle as o
    rp = shard.row_ptr.numpy()
    r0, r1 = rows if rows is not None else (0, shard.rows)
    Y = o.spmm_csr(rp, shard.cols_for(layout).numpy(), shard.val.numpy(), X.numpy(), r0, r1)
    out.copy_(torch.from_numpy(Y))
    return out


def _worker(rank, world, port, case, K, result_q, group_floats=128, staging=False,
            output="replicated", autotune=False, balance="nnz", engine="oracle", row_chunks=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as o
        n = int(case["n"])
        rp, ci, va = o.coo_to_csr(n, n, case["rows"], case["cols"], case["vals"])
        shard = make_shard(rp, ci, va, rank, world, "cpu", balance=balance)
        # engine "product": the default spmm_fn, i.e. the library's CPU twin
        prop = RowPartitionedPropagator(shard, spmm_fn=_oracle_spmm if engine == "oracle" else None,
                                        group_floats=group_floats, host_staging=staging,
                                        row_chunks=row_chunks)
        X0 = torch.from_numpy(case["X"])
        tuned = None
        if autotune:
            times = prop.autotune(X0, K, output=output, candidates=(8, 64, 16, 0, "r3"), reps=1)
            assert sorted(times, key=str) == sorted([8, 16, 64, 0, "r3"], key=str)
            tuned = (prop.group_floats, prop.row_chunks)
        out = prop.propagate(X0, K, output=output)
        res = (out.numpy(), shard.bounds)
        result_q.put((rank, res) if not autotune else (rank, (res, tuned)))
    finally:
        dist.destroy_process_group()


def _check_results(results, case, K, world, output, name):
    want = case[f"Y{K}"]
    for r in range(world):
        got, rb = results[r]
        w = want if output == "replicated" else want[rb[r]:rb[r + 1]]
        assert got.shape == w.shape, (name, r)
        assert np.array_equal(got.view(np.uint32), w.view(np.uint32)), (name, r)


@pytest.mark.parametrize("world,name,K,gf,staging,output,balance,engine", [
    (2, "norm_n48_F65", 2, 128, False, "replicated", "nnz", "oracle"),
    (2, "hub1000_F65", 2, 16, False, "sharded", "nnz", "oracle"),
    (3, "norm_n48_F602", 3, 128, False, "replicated", "rows", "oracle"),
    (3, "norm_n48_F602", 2, 128, False, "sharded", "nnz", "product"),
    (4, "raw_unsorted_dups_F7", 3, 2, False, "replicated", "nnz", "product"),
    (4, "raw_unsorted_dups_F7", 1, 2, False, "sharded", "rows", "oracle"),
    (2, "isolated_F17", 1, 4, True, "replicated", "nnz", "oracle"),
    (2, "norm_n48_F130", 2, 64, True, "sharded", "nnz", "product"),
    (3, "hub1000_F130", 2, 64, False, "replicated", "nnz", "product"),
    (4, "hub1000_F65", 2, 32, False, "sharded", "rows", "product"),
    (3, "hub1000_F65", 2, 0, False, "replicated", "nnz", "product:rc4"),
    (2, "norm_n48_F602", 2, 0, False, "sharded", "nnz", "oracle:rc3"),
    (4, "raw_unsorted_dups_F7", 3, 0, True, "sharded", "rows", "product:rc2")])
def test_row_partition_gloo_bit_exact(tiny_cases, oracle, world, name, K, gf, staging, output,
                                      balance, engine):
    case = tiny_cases[name]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    eng, _, rc = engine.partition(":rc")
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, K, q, gf, staging, output,
                                               False, balance, eng, int(rc or 1)))
             for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    _check_results(results, case, K, world, output, name)


@pytest.mark.parametrize("output", ["sharded", "replicated"])
def test_row_partition_autotune_gloo(tiny_cases, oracle, output):
    """autotune() times each group width collectively: every rank must pick
    the same width (the all-gathers' shapes depend on it) and the result stays
    bit-exact."""
    case, K, world = tiny_cases["norm_n48_F65"], 2, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, K, q, 128, False, output,
                                               True)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len({got[r][1] for r in range(world)}) == 1
    _check_results({r: got[r][0] for r in range(world)}, case, K, world, output, "autotune")


def _tiled_worker(rank, world, port, case, K, C, result_q, staging, engine):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as o
        from sgc_amd.distributed import TiledPropagator
        n = int(case["n"])
        rp, ci, va = o.coo_to_csr(n, n, case["rows"], case["cols"], case["vals"])
        tp = TiledPropagator(rp, ci, va, rank, world, C, "cpu", group_floats=8,
                             host_staging=staging,
                             spmm_fn=_oracle_spmm if engine == "oracle" else None)
        X0 = torch.from_numpy(case["X"])
        out = tp.propagate(X0, K, output="sharded")
        out2 = tp.propagate(X0, K, output="sharded")  # buffers reused
        assert torch.equal(out, out2)
        result_q.put((rank, (out.numpy(), np.repeat(tp.shard.bounds, 1))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,C,name,K,staging,engine", [
    (4, 2, "norm_n48_F602", 2, False, "product"), (2, 2, "norm_n48_F65", 3, False, "oracle"),
    (4, 4, "hub1000_F65", 2, False, "product"), (4, 2, "raw_unsorted_dups_F7", 2, True, "oracle"),
    (6, 3, "norm_n48_F130", 2, False, "product")])
def test_tiled_partition_gloo_bit_exact(tiny_cases, oracle, world, C, name, K, staging, engine):
    """2-D partition (row blocks x feature blocks): every rank's full-width
    row block of X_K equals the reference's rows, bit for bit."""
    case = tiny_cases[name]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tiled_worker, args=(r, world, port, case, K, C, q, staging,
                                                     engine)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = case[f"Y{K}"]
    R = world // C
    for r in range(world):
        arr, rb = got[r]
        i = r // C
        w = want[rb[i]:rb[i + 1]]
        assert arr.shape == w.shape and np.array_equal(arr.view(np.uint32), w.view(np.uint32)), r
    del R


def test_gathered_layout():
    """nnz-balanced blocks of unequal rows: node j sits at row p*B + (j - r_p)
    of the gathered buffer; equal blocks are the identity."""
    from sgc_amd.distributed import gathered_index
    rp = np.array([0, 100, 101, 102, 103, 203, 204, 205, 305])
    b = nnz_balanced_bounds(rp, 3)
    B = int(np.max(np.diff(b)))
    g = gathered_index(b, B, np.arange(8))
    for p in range(3):
        for j in range(b[p], b[p + 1]):
            assert g[j] == p * B + j - b[p]
    assert len(set(g.tolist())) == 8
    eb = equal_row_bounds(10, 4)
    assert np.array_equal(gathered_index(eb, 3, np.arange(10)), np.arange(10))
    sh = make_shard(np.arange(11), np.arange(10), np.ones(10, np.float32), 1, 4, "cpu",
                    balance="rows")
    assert sh.identity_layout and sh.col_gathered is sh.col_idx


@pytest.mark.parametrize("name", ["hub1000_F130", "norm_n48_F65", "isolated_F17",
                                  "raw_unsorted_dups_F7"])
def test_make_shard_device_matches_host(tiny_cases, name):
    """The shards the multi-GPU call builds from the adjacency's own arrays
    (make_shard_device: no host copy of S) equal the host slicing's, bounds,
    row_ptr, both column-id arrays and values, for every rank at P = 1..8."""
    from sgc_amd.distributed import make_shard_device
    from sgc_amd.propagate import csr_of
    c = tiny_cases[name]
    n = int(c["n"])
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.stack([c["rows"], c["cols"]])),
                                  torch.from_numpy(c["vals"]), (n, n))
    csr = csr_of(adj)
    rp, ci, va = (t.numpy() for t in (csr.row_ptr, csr.col_idx, csr.val))
    for world in range(1, 9):
        for rank in range(world):
            h = make_shard(rp, ci, va, rank, world, "cpu")
            d = make_shard_device(csr, rank, world)
            assert np.array_equal(h.bounds, d.bounds), (world, rank)
            for f in ("row_ptr", "col_idx", "val", "col_gathered"):
                assert torch.equal(getattr(h, f), getattr(d, f)), (world, rank, f)
            assert d.n == h.n and d.block == h.block


# ---------------------------------------------------------------------------
# Cyclic row tiles + column-ordered exchange (CyclicRowPropagator).

def test_cyclic_layout_and_split():
    """Tiles dealt round-robin: every global row is owned once, local rows are
    ascending, the exchange-buffer map is a bijection that sends column group
    g to rows [g*P*Tg*b, (g+1)*P*Tg*b), and each row's group CSRs concatenate
    to its full CSR-ordered row."""
    from sgc_amd.distributed import cyclic_gathered_index, cyclic_layout, make_cyclic_shard
    from oracle import oracle as o
    rng = np.random.default_rng(3)
    n, P, b, G = 103, 3, 4, 3
    Tg, T = cyclic_layout(n, P, b, G)
    assert T == G * Tg and P * T * b >= n
    rows = rng.integers(0, n, 900)
    cols = rng.integers(0, n, 900)
    key = np.unique(rows * n + cols)  # canonical CSR: rows sorted by column
    rows, cols = key // n, key % n
    rp, ci, va = o.coo_to_csr(n, n, rows, cols, rng.standard_normal(key.size).astype(np.float32))
    owned = []
    for r in range(P):
        sh = make_cyclic_shard(rp, ci, va, r, P, "cpu", tile=b, groups=G)
        gr = sh.global_rows[:sh.n_valid]
        assert np.all(np.diff(gr) > 0) and np.all(sh.global_rows[sh.n_valid:] >= n)
        owned.append(gr)
        in_rp = sh.csr_input.row_ptr.numpy()
        for i, j in enumerate(gr):
            full = ci[rp[j]:rp[j + 1]]
            parts, vparts = [], []
            for g in range(G):
                s_rp = sh.sub[g].row_ptr.numpy()
                k0, k1 = s_rp[i], s_rp[i + 1]
                c = sh.sub[g].col_idx.numpy()[k0:k1]
                lo, hi = g * P * Tg * b, (g + 1) * P * Tg * b
                assert np.all((c >= lo) & (c < hi))
                parts.append(c)
                vparts.append(sh.sub[g].val.numpy()[k0:k1])
            assert np.array_equal(np.concatenate(parts), cyclic_gathered_index(full, P, b, Tg))
            assert np.array_equal(np.concatenate(vparts), va[rp[j]:rp[j + 1]])
            assert np.array_equal(sh.csr_input.col_idx.numpy()[in_rp[i]:in_rp[i + 1]], full)
    assert np.array_equal(np.sort(np.concatenate(owned)), np.arange(n))
    m = cyclic_gathered_index(np.arange(P * T * b), P, b, Tg)
    assert np.array_equal(np.sort(m), np.arange(P * T * b))


def test_cyclic_rejects_rows_out_of_group_order():
    """A storage-order row that returns to an earlier column group cannot be
    split into ordered passes: refused loudly, fine with one group."""
    from sgc_amd.distributed import make_cyclic_shard
    rp = np.array([0, 3, 3, 3, 3], dtype=np.int64)
    ci = np.array([3, 0, 1], dtype=np.int32)  # row 0: group 1, then group 0
    va = np.ones(3, np.float32)
    with pytest.raises(ValueError, match="column-group order"):
        make_cyclic_shard(rp, ci, va, 0, 2, "cpu", tile=1, groups=2)
    make_cyclic_shard(rp, ci, va, 0, 2, "cpu", tile=1, groups=1)


def _cyclic_worker(rank, world, port, case, K, result_q, tile, groups, staging, output):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as o
        from sgc_amd.distributed import CyclicRowPropagator
        n = int(case["n"])
        rp, ci, va = o.coo_to_csr(n, n, case["rows"], case["cols"], case["vals"])
        cp = CyclicRowPropagator(rp, ci, va, rank, world, "cpu", tile=tile, groups=groups,
                                 host_staging=staging)
        X0 = torch.from_numpy(case["X"])
        out = cp.propagate(X0, K, output=output)
        out2 = cp.propagate(X0, K, output=output)  # buffers reused
        assert torch.equal(out, out2)
        result_q.put((rank, (out.numpy(), cp.row_index)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,name,K,tile,groups,staging,output", [
    (2, "norm_n48_F65", 2, 4, 3, False, "sharded"),
    (3, "norm_n48_F602", 3, 2, 4, False, "replicated"),
    (4, "hub1000_F65", 2, 16, 4, False, "sharded"),
    (3, "hub1000_F130", 2, 8, 2, True, "sharded"),
    (4, "raw_unsorted_dups_F7", 2, 1, 1, False, "replicated"),  # unsorted rows: one group
    (2, "isolated_F17", 1, 4, 2, False, "replicated"),
    (4, "norm_n48_F130", 2, 64, 1, False, "sharded")])  # one tile per rank: empty ranks
def test_cyclic_partition_gloo_bit_exact(tiny_cases, world, name, K, tile, groups, staging,
                                         output):
    """Every rank's rows of X_K (column-group passes chained with
    SPMM_ACCUMULATE through the product CPU twin) equal the reference's rows
    bit for bit; replicated output equals all of it."""
    case = tiny_cases[name]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cyclic_worker, args=(r, world, port, case, K, q, tile, groups,
                                                      staging, output)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = case[f"Y{K}"]
    seen = []
    for r in range(world):
        arr, ri = got[r]
        w = want if output == "replicated" else want[ri]
        assert arr.shape == w.shape and np.array_equal(arr.view(np.uint32), w.view(np.uint32)), r
        seen.append(ri)
    assert np.array_equal(np.sort(np.concatenate(seen)), np.arange(int(case["n"])))


# ---------------------------------------------------------------------------
# Feature (column) partition: no exchange between hops, one chunked all-gather.

def test_feature_bounds():
    b, B = feature_bounds(602, 8)
    assert B == 76 and b.tolist() == [0, 76, 152, 228, 304, 380, 456, 532, 602]
    b, B = feature_bounds(602, 2)
    assert B == 304 and b.tolist() == [0, 304, 602]
    b, B = feature_bounds(5, 4)  # more ranks than aligned blocks: empty tails
    assert B == 4 and b.tolist() == [0, 4, 5, 5, 5]
    b, B = feature_bounds(7, 3, align=1)
    assert B == 3 and b.tolist() == [0, 3, 6, 7]


def test_row_chunks():
    assert row_chunks(10, 4) == [(0, 3), (3, 6), (6, 9), (9, 10)]
    assert row_chunks(3, 8) == [(0, 1), (1, 2), (2, 3)]
    assert row_chunks(0, 4) == [(0, 0)]


def _feature_worker(rank, world, port, case, K, result_q, chunks, align, staging, output,
                    exchange="auto", pieces=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as o
        n = int(case["n"])
        rp, ci, va = o.coo_to_csr(n, n, case["rows"], case["cols"], case["vals"])

        def spmm_fn(X, r0, r1, out):
            out.copy_(torch.from_numpy(o.spmm_csr(rp, ci, va, X.numpy(), r0, r1)))

        prop = FeaturePartitionedPropagator(spmm_fn=spmm_fn, chunks=chunks, align=align,
                                            host_staging=staging, exchange=exchange,
                                            pieces=pieces)
        out = prop.propagate(torch.from_numpy(case["X"]), K, output=output)
        out2 = prop.propagate(torch.from_numpy(case["X"]), K, output=output)  # buffers reused
        assert torch.equal(out, out2)
        result_q.put((rank, (out.numpy(), equal_row_bounds(n, world))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,name,K,chunks,align,staging,output", [
    (2, "norm_n48_F602", 2, 4, 4, False, "replicated"), (2, "norm_n48_F602", 2, 4, 4, False, "sharded"),
    (3, "norm_n48_F65", 3, 3, 4, False, "replicated"), (3, "norm_n48_F65", 2, 3, 4, False, "sharded"),
    (4, "hub1000_F130", 2, 2, 4, False, "replicated"),
    (4, "raw_unsorted_dups_F7", 3, 5, 1, False, "sharded"),
    (2, "isolated_F17", 1, 1, 2, True, "replicated"), (3, "norm_n48_F3", 2, 4, 1, True, "sharded")])
@pytest.mark.parametrize("exchange,pieces", [("auto", None), ("alltoall", None), ("pairwise", 3)])
def test_feature_partition_gloo_bit_exact(tiny_cases, oracle, world, name, K, chunks, align,
                                          staging, output, exchange, pieces):
    """Sharded output: the all-to-all after the last hop, or the pairwise
    exchange overlapped with it (auto = pairwise at world 2), k row pieces
    per destination (3 pieces of 16-row blocks: uneven and empty pieces)."""
    if output == "replicated" and exchange != "auto":
        pytest.skip("the exchange mode applies to sharded output")
    case = tiny_cases[name]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_feature_worker,
                         args=(r, world, port, case, K, q, chunks, align, staging, output,
                               exchange, pieces))
             for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    _check_results(results, case, K, world, output, name)


# ---------------------------------------------------------------------------
# Line partition: whole 128-B lines per rank + a row-sharded tail.

def test_line_bounds():
    assert line_bounds(602, 8) == (64, 512)    # 19 lines: 2 per rank + 3 tail lines
    assert line_bounds(602, 4) == (128, 512)   # 4 per rank + 3
    assert line_bounds(602, 2) == (288, 576)   # 9 per rank + 1 (26 floats)
    assert line_bounds(602, 19) == (32, 602)   # every line its rank's, the last short
    assert line_bounds(65, 4) == (0, 0)        # fewer lines than ranks: all tail
    assert line_bounds(64, 2) == (32, 64)      # no tail
    assert line_bounds(7, 1) == (32, 7)


def _line_worker(rank, world, port, case, K, result_q, chunks, staging, output, balance):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as o
        n = int(case["n"])
        rp, ci, va = o.coo_to_csr(n, n, case["rows"], case["cols"], case["vals"])

        def main_fn(X, r0, r1, out):
            out.copy_(torch.from_numpy(o.spmm_csr(rp, ci, va, X.numpy(), r0, r1)))

        shard = make_shard(rp, ci, va, rank, world, "cpu", balance=balance)
        prop = LinePartitionedPropagator(shard, main_spmm_fn=main_fn, tail_spmm_fn=_oracle_spmm,
                                         chunks=chunks, host_staging=staging)
        X0 = torch.from_numpy(case["X"])
        out = prop.propagate(X0, K, output=output)
        out2 = prop.propagate(X0, K, output=output)  # buffers reused
        assert torch.equal(out, out2)
        result_q.put((rank, (out.numpy(), equal_row_bounds(n, world))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,name,K,chunks,staging,output,balance", [
    (2, "norm_n48_F602", 2, 4, False, "replicated", "nnz"),   # 9 lines each + a 26-float tail
    (2, "norm_n48_F602", 3, 2, False, "sharded", "nnz"),
    (4, "norm_n48_F602", 2, 3, False, "replicated", "rows"),  # 4 lines each + 90-float tail
    (3, "hub1000_F130", 2, 2, False, "sharded", "nnz"),       # 1 line each + 34-float tail
    (4, "hub1000_F130", 2, 4, True, "replicated", "nnz"),     # 1 line each + 2-float tail
    (3, "norm_n48_F65", 2, 3, False, "replicated", "nnz"),    # a line each (the last 1 float), no tail
    (4, "raw_unsorted_dups_F7", 3, 5, False, "sharded", "nnz"),  # all tail
    (2, "isolated_F17", 1, 1, True, "replicated", "nnz"),
    (2, "norm_n48_F3", 2, 4, False, "sharded", "rows"),
    (8, "norm_n48_F602", 2, 4, False, "replicated", "nnz"),    # the P = 8 layout: 64 + 90-float tail
    (8, "hub1000_F130", 2, 3, False, "sharded", "nnz")])       # 5 lines over 8 ranks: all tail
def test_line_partition_gloo_bit_exact(tiny_cases, oracle, world, name, K, chunks, staging,
                                       output, balance):
    """Main line blocks need no exchange; the tail's row blocks are gathered
    after every hop and read through the gathered column ids (uneven nnz
    blocks, so the gathered layout is not the identity)."""
    case = tiny_cases[name]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_line_worker,
                         args=(r, world, port, case, K, q, chunks, staging, output, balance))
             for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    _check_results(results, case, K, world, output, name)


# ---------------------------------------------------------------------------
# Data-parallel classifier over row shards (ShardedSGCTrainer).

def _trainer_worker(rank, world, port, result_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sgc_amd.distributed import ShardedSGCTrainer, _torch_loss_grad
        from sgc_amd.models import SGC
        g = torch.Generator().manual_seed(0)
        n, F, C = 97, 13, 5
        X = torch.randn(n, F, generator=g)
        y = torch.randint(0, C, (n,), generator=g)
        train = torch.arange(0, n, 2)  # every other row trains
        rb = equal_row_bounds(n, world)
        r0, r1 = int(rb[rank]), int(rb[rank + 1])
        mask = (train >= r0) & (train < r1)
        Xl, yl = X[train[mask]], y[train[mask]]
        torch.manual_seed(1)
        model = SGC(F, C)
        tr = ShardedSGCTrainer(model, loss_grad_fn=_torch_loss_grad)
        loss0 = tr.loss(Xl, yl, train.numel())
        g0 = (float(loss0), model.W.weight.grad.numpy().copy(), model.W.bias.grad.numpy().copy())
        opt = torch.optim.LBFGS(model.parameters(), lr=1)

        def closure():
            opt.zero_grad()
            return tr.loss(Xl, yl, train.numel())
        for _ in range(2):
            opt.step(closure)
        result_q.put((rank, g0, model.W.weight.detach().numpy().copy(),
                      model.W.bias.detach().numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_trainer_matches_single_process_lbfgs(world):
    """reddit.py:51-64's LBFGS closure, data-parallel over row shards, ends at
    the single-process weights (fp32 tolerance: the reduction order differs)."""
    from sgc_amd.models import SGC
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_trainer_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict((r, (w, b, g0)) for r, g0, w, b in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = torch.Generator().manual_seed(0)
    n, F, C = 97, 13, 5
    X = torch.randn(n, F, generator=g)
    y = torch.randint(0, C, (n,), generator=g)
    train = torch.arange(0, n, 2)
    torch.manual_seed(1)
    model = SGC(F, C)
    opt = torch.optim.LBFGS(model.parameters(), lr=1)

    def closure():
        opt.zero_grad()
        z = X[train] @ model.W.weight.t() + model.W.bias
        loss = torch.nn.functional.cross_entropy(z, y[train])
        loss.backward()
        return loss
    loss0 = closure()
    want0 = (float(loss0), model.W.weight.grad.numpy().copy(), model.W.bias.grad.numpy().copy())
    for _ in range(2):
        opt.step(closure)
    for r in range(world):
        w, b, g0 = results[r]
        # one closure: global mean loss and gradients (fp32 tolerance)
        assert abs(g0[0] - want0[0]) <= 1e-6 * max(1.0, abs(want0[0]))
        np.testing.assert_allclose(g0[1], want0[1], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(g0[2], want0[2], rtol=1e-5, atol=1e-6)
        # two LBFGS steps (lr=1 amplifies rounding differences: looser)
        np.testing.assert_allclose(w, model.W.weight.detach().numpy(), rtol=5e-3, atol=1e-4)
        np.testing.assert_allclose(b, model.W.bias.detach().numpy(), rtol=5e-3, atol=1e-4)
        assert np.array_equal(w, results[0][0])  # identical on every rank


def _ipc_agreement_worker(rank, world, port, fail_rank, test_fail_rank, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sgc_amd.distributed as D

        class FakePeers:
            closed = False

            def __init__(self, group, rank_, world_, n, ld, device):
                if rank_ == fail_rank:
                    raise RuntimeError("no IPC here")

            def self_test(self):
                return rank != test_fail_rank

            def close(self):
                FakePeers.closed = True

        D.IpcPeers = FakePeers

        class Prop:
            pass
        prop = Prop()
        ipc = D._ipc_for(prop, dist.group.WORLD, rank, world, 10, 32, torch.device("cpu"))
        again = D._ipc_for(prop, dist.group.WORLD, rank, world, 10, 32, torch.device("cpu"))
        q.put((rank, ipc is not None, again is ipc, getattr(prop, "ipc_unavailable", None)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fail_rank,test_fail_rank", [(-1, -1), (0, -1), (-1, 1), (2, 0)])
def test_ipc_window_is_all_or_none(fail_rank, test_fail_rank):
    """The IPC exchange is used by every rank or by none: a rank that cannot
    map its peers (or whose set-up self-test reads a wrong value) makes the
    whole group keep the collective path -- a MIN all-reduce of the outcome --
    and the decision is cached on the propagator (one set-up per shape)."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ipc_agreement_worker,
                         args=(r, world, port, fail_rank, test_fail_rank, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, rest) for r, *rest in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = fail_rank < 0 and test_fail_rank < 0
    for r in range(world):
        used, cached, why = got[r]
        assert used == want and cached, (r, got[r])
        assert (why is None) == want, (r, why)
