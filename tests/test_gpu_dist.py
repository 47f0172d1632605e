"""The row-partitioned path over RCCL (backend "nccl") on the one GPU a test
box has: world size 1 exercises process-group init with device_id, the async
all_gather_into_tensor per feature group, the stream waits, the 128-B padded
layout and the final compaction -- bit-exact against the reference goldens.
World sizes 2-4 of the same class run over gloo in tests/test_distributed.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def nccl_group():
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0",
                      WORLD_SIZE="1")
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("pad_input", [None, False])
@pytest.mark.parametrize("output", ["replicated", "sharded"])
@pytest.mark.parametrize("name,K,gf", [("norm_n48_F602", 2, 128), ("hub1000_F130", 2, 64),
                                       ("norm_n48_F65", 3, 32), ("isolated_F17", 1, 128),
                                       ("norm_n48_F602", 3, 320)])
def test_rccl_row_partition_bit_exact(nccl_group, tiny_cases, oracle, name, K, gf, output,
                                      pad_input):
    """pad_input=False: hop 1 reads the caller's 8-B aligned rows directly and
    the last feature group is narrower than its exchange buffer (the P >= 8
    default)."""
    from sgc_amd.distributed import RowPartitionedPropagator, make_shard
    c = tiny_cases[name]
    n = int(c["n"])
    rp, ci, va = oracle.coo_to_csr(n, n, c["rows"], c["cols"], c["vals"])
    shard = make_shard(rp, ci, va, 0, 1, "cuda")
    prop = RowPartitionedPropagator(shard, group_floats=gf, pad_input=pad_input)
    out = prop.propagate(torch.from_numpy(c["X"]).cuda(), K, output=output)
    torch.cuda.synchronize()
    want = c[f"Y{K}"]
    assert out.shape == want.shape
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want.view(np.uint32))
    out2 = prop.propagate(torch.from_numpy(c["X"]).cuda(), K, output=output)  # buffers reused
    assert torch.equal(out, out2)


@pytest.mark.parametrize("output", ["replicated", "sharded"])
@pytest.mark.parametrize("name,K,chunks", [("norm_n48_F602", 2, 4), ("hub1000_F130", 2, 3),
                                           ("norm_n48_F65", 3, 1), ("isolated_F17", 1, 2),
                                           ("special_values_F11", 2, 5)])
def test_rccl_feature_partition_bit_exact(nccl_group, tiny_cases, oracle, name, K, chunks, output):
    """The feature-partitioned path end to end on the HIP kernels + RCCL: the
    column-block copy, local hops, chunked last hop, async all-gather and the
    unpack into [N, F]."""
    from sgc_amd.distributed import FeaturePartitionedPropagator
    from sgc_amd.propagate import DeviceCSR
    c = tiny_cases[name]
    n = int(c["n"])
    rp, ci, va = oracle.coo_to_csr(n, n, c["rows"], c["cols"], c["vals"])
    csr = DeviceCSR.from_host_arrays(rp, ci, va, device="cuda")
    prop = FeaturePartitionedPropagator(csr, chunks=chunks)
    out = prop.propagate(torch.from_numpy(c["X"]).cuda(), K, output=output)
    torch.cuda.synchronize()
    want = c[f"Y{K}"]
    assert out.shape == want.shape
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want.view(np.uint32))
    out2 = prop.propagate(torch.from_numpy(c["X"]).cuda(), K, output=output)
    assert torch.equal(out, out2)


def test_feature_partition_rank_work_pubmed():
    """What rank 0 and rank 7 of 8 compute at Pubmed shape -- K=2 hops on a
    64-column block over all rows, chunked last hop -- equals those columns of
    the single-GPU result (itself pinned to the reference's hash elsewhere)."""
    from sgc_amd import graphs
    from sgc_amd.distributed import feature_bounds
    from sgc_amd.propagate import DeviceCSR, propagate, spmm
    S = graphs.synthetic_graph("pubmed", seed=0)
    X = torch.from_numpy(graphs.synthetic_features("pubmed", S.n, 500, seed=1)).cuda()
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device="cuda")
    full = propagate(csr, X, 2)
    bounds, B = feature_bounds(500, 8)
    for p in (0, 7):
        c0, c1 = int(bounds[p]), int(bounds[p + 1])
        a = X[:, c0:c1].contiguous()
        h1 = spmm(csr, a)
        h2 = torch.cat([spmm(csr, h1, r0, min(S.n, r0 + 5000)) for r0 in range(0, S.n, 5000)])
        assert torch.equal(h2, full[:, c0:c1])


def test_rccl_sharded_trainer_fused_kernel(nccl_group):
    """ShardedSGCTrainer on the fused HIP loss/gradient kernel + RCCL
    all-reduce: the global mean loss and gradients equal torch's."""
    from sgc_amd.distributed import ShardedSGCTrainer
    from sgc_amd.models import SGC
    g = torch.Generator().manual_seed(0)
    X = torch.randn(3001, 602, generator=g).cuda()
    y = torch.randint(0, 41, (3001,), generator=g).cuda()
    torch.manual_seed(2)
    model = SGC(602, 41).cuda()
    tr = ShardedSGCTrainer(model)
    loss = tr.loss(X, y, 3001)
    gw, gb = model.W.weight.grad.clone(), model.W.bias.grad.clone()
    Xd, Wd, bd = X.double(), model.W.weight.detach().double(), model.W.bias.detach().double()
    Wd.requires_grad_(True)
    bd.requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(Xd @ Wd.t() + bd, y)
    ref.backward()
    assert abs(loss.item() - ref.item()) <= 1e-5 * abs(ref.item())
    torch.testing.assert_close(gw.double(), Wd.grad, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(gb.double(), bd.grad, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("pad_input", [None, False])
@pytest.mark.parametrize("output", ["replicated", "sharded"])
@pytest.mark.parametrize("name,K,tile,groups", [("norm_n48_F602", 2, 4, 3), ("hub1000_F130", 2, 16, 4),
                                                ("norm_n48_F65", 3, 1, 5), ("isolated_F17", 1, 8, 2),
                                                ("norm_n48_F602", 3, 64, 1)])
def test_cyclic_partition_world1_bit_exact(tiny_cases, oracle, name, K, tile, groups, output,
                                           pad_input):
    """CyclicRowPropagator on the GPU: hop >= 2 as column-group passes chained
    by SGC_SPMM_ACCUMULATE, the last pass in row chunks each handed to the
    exchange (a copy at world 1), the replicated output's re-ordering."""
    from sgc_amd.distributed import CyclicRowPropagator
    c = tiny_cases[name]
    n = int(c["n"])
    rp, ci, va = oracle.coo_to_csr(n, n, c["rows"], c["cols"], c["vals"])
    cp = CyclicRowPropagator(rp, ci, va, 0, 1, "cuda", tile=tile, groups=groups,
                             pad_input=pad_input)
    X0 = torch.from_numpy(c["X"]).cuda()
    out = cp.propagate(X0, K, output=output)
    torch.cuda.synchronize()
    want = c[f"Y{K}"] if output == "replicated" else c[f"Y{K}"][cp.row_index]
    assert out.shape == want.shape
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want.view(np.uint32))
    out2 = cp.propagate(X0, K, output=output)  # prepared launches replayed
    assert torch.equal(out, out2)


@pytest.mark.slow
@pytest.mark.parametrize("groups", [4, 8])
def test_cyclic_partition_reddit_shape_hash(shapes_golden, groups):
    """Full Reddit shape through the column-group passes (world 1): the
    reference's X_2 hash."""
    import hashlib
    from sgc_amd import graphs
    from sgc_amd.distributed import CyclicRowPropagator
    g = shapes_golden["reddit"]
    S = graphs.synthetic_graph("reddit", seed=g["seed"])
    X = graphs.synthetic_features("reddit", g["n"], g["features"], seed=g["feature_seed"])
    cp = CyclicRowPropagator(S.row_ptr, S.col_idx, S.val, 0, 1, "cuda", tile=64, groups=groups)
    out = cp.propagate(torch.from_numpy(X).cuda(), 2, output="replicated")
    torch.cuda.synchronize()
    assert hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest() == g["outputs"]["2"]["sha"]


@pytest.mark.parametrize("shape,P,K", [("pubmed", 8, 2), ("pubmed", 3, 3), ("cora", 8, 2)])
def test_feature_partition_rank_steps_gpu(shape, P, K):
    """Every rank's step of the feature partition on the HIP kernels (the
    exchange replaced by capturing the all-to-all's send buffer): hop 1 in
    place on the caller's block when it is 16-B laned (Pubmed's 64/52 and
    168/164-column blocks, Cora's 180), through the compact copy otherwise
    (Cora's last, 173 columns), pad-flagged hops in the engine's buffers, the one-launch
    last hop laid out by destination -- equal to those columns and rows of the
    single-GPU result (pinned to the reference's hashes elsewhere)."""
    from sgc_amd import graphs
    from sgc_amd.distributed import (FeaturePartitionedPropagator, equal_row_bounds,
                                     feature_bounds)
    from sgc_amd.propagate import DeviceCSR, propagate

    class Capture(FeaturePartitionedPropagator):
        def _all_to_all(self, recv, send):
            self.sent = send.clone()
            recv.copy_(send)
            return None

    S = graphs.synthetic_graph(shape, seed=0)
    F = graphs.SHAPES[shape]["features"]
    X = torch.from_numpy(graphs.synthetic_features(shape, S.n, F, seed=1)).cuda()
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device="cuda")
    full = propagate(csr, X, K)
    fb, B = feature_bounds(F, P)
    rb = equal_row_bounds(S.n, P)
    Bn = -(-S.n // P)
    for p in range(P):
        c0, c1 = int(fb[p]), int(fb[p + 1])
        prop = Capture(csr, rank=p, world_size=P)
        for _ in range(2):  # buffers reused
            prop.propagate(X, K, output="sharded")
            torch.cuda.synchronize()
            for q in range(P):
                r0, r1 = int(rb[q]), int(rb[q + 1])
                got = prop.sent[q * Bn:q * Bn + (r1 - r0), :c1 - c0]
                assert torch.equal(got, full[r0:r1, c0:c1]), (p, q)
