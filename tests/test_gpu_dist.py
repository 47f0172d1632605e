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


@pytest.mark.parametrize("name,K,gf", [("norm_n48_F602", 2, 128), ("hub1000_F130", 2, 64),
                                       ("norm_n48_F65", 3, 32), ("isolated_F17", 1, 128)])
def test_rccl_row_partition_bit_exact(nccl_group, tiny_cases, oracle, name, K, gf):
    from sgc_amd.distributed import RowPartitionedPropagator, make_shard
    c = tiny_cases[name]
    n = int(c["n"])
    rp, ci, va = oracle.coo_to_csr(n, n, c["rows"], c["cols"], c["vals"])
    shard = make_shard(rp, ci, va, 0, 1, "cuda")
    prop = RowPartitionedPropagator(shard, group_floats=gf)
    out = prop.propagate(torch.from_numpy(c["X"]).cuda(), K)
    torch.cuda.synchronize()
    want = c[f"Y{K}"]
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want.view(np.uint32))
    out2 = prop.propagate(torch.from_numpy(c["X"]).cuda(), K)  # buffers reused
    assert torch.equal(out, out2)
