"""The multi-GPU paths on the one GPU a test box has, bit-exact.

* the native multi-device engine (sgc_mgpu_*, csrc/mgpu.hip) with VIRTUAL
  devices -- the same index repeated: every entry its own stream, buffers and
  column block, exactly the code an 8-GPU node runs minus the xGMI hops;
* the unchanged `sgc_precompute` under torchrun (2 ranks sharing the GPU over
  gloo: the group is initialised by the drop-in from torchrun's environment),
  and the reddit driver run that way end to end;
* `bench.py --gpus 2` launching its own ranks (what the driver's scaling run
  does when it does not use torchrun itself);
* the P = 8 partitions at FULL BASELINE size (8 gloo ranks on the GPU, the
  product propagators, X_K assembled from every rank's rows) against the
  reference's own hashes: Reddit K = 2 for the row, cyclic, feature and 2-D
  tile partitions, RMAT K = 3 for the row partition.
"""
import hashlib
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _torchrun(nproc, script_args, env_extra=None, timeout=600):
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.update(env_extra or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", *script_args]
    return subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True,
                          timeout=timeout)


def _last_json(text):
    for line in reversed(text.strip().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise AssertionError(f"no JSON line in output:\n{text[-2000:]}")


def _csr(case, oracle):
    from sgc_amd.propagate import DeviceCSR
    n = int(case["n"])
    rp, ci, va = oracle.coo_to_csr(n, n, case["rows"], case["cols"], case["vals"])
    return DeviceCSR.from_host_arrays(rp, ci, va, device="cuda")


# ---------------------------------------------------------------------------
# native multi-device engine, virtual devices

@pytest.mark.parametrize("ndev", [2, 3, 8])
@pytest.mark.parametrize("name,K", [("norm_n48_F602", 2), ("hub1000_F130", 2),
                                    ("norm_n48_F65", 3), ("isolated_F17", 1),
                                    ("raw_unsorted_dups_F7", 3), ("special_values_F11", 2),
                                    ("no_edges_F5", 2), ("norm_n48_F3", 3)])
def test_mgpu_engine_virtual_devices_bit_exact(tiny_cases, oracle, ndev, name, K):
    """Feature blocks over ndev virtual devices (some empty when F < 4 ndev),
    pulled from the home device, K local hops, the last one stored into the
    caller's X_K: equal to the reference's X_K bit for bit, twice (buffers
    and plans reused)."""
    from sgc_amd.multigpu import DeviceSet
    case = tiny_cases[name]
    csr = _csr(case, oracle)
    X = torch.from_numpy(case["X"]).cuda()
    ds = DeviceSet.get([0] * ndev)
    want = case[f"Y{K}"]
    for _ in range(2):
        out = torch.full(X.shape, float("nan"), device="cuda")
        ds.propagate(csr, X, K, out)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().view(np.uint32), want.view(np.uint32))


def test_mgpu_engine_strided_input_and_output(tiny_cases, oracle):
    """X_0 a column view of a wider tensor, X_K written into a column view:
    no byte outside the view changes (the last hop never pad-writes Y)."""
    from sgc_amd.multigpu import DeviceSet
    case = tiny_cases["norm_n48_F130"]
    csr = _csr(case, oracle)
    n, F = case["X"].shape
    big = torch.randn(n, F + 7, device="cuda")
    big[:, 3:3 + F] = torch.from_numpy(case["X"]).cuda()
    dst = torch.full((n, F + 9), 7.0, device="cuda")
    DeviceSet.get([0, 0, 0, 0]).propagate(csr, big[:, 3:3 + F], 2, dst[:, 5:5 + F])
    torch.cuda.synchronize()
    got = dst.cpu().numpy()
    assert np.array_equal(got[:, 5:5 + F].view(np.uint32), case["Y2"].view(np.uint32))
    assert (got[:, :5] == 7.0).all() and (got[:, 5 + F:] == 7.0).all()


def test_sgc_precompute_with_device_set_env(tiny_cases, oracle, monkeypatch):
    """SGC_AMD_DEVICES routes the unchanged call through the engine."""
    from sgc_amd.utils import sgc_precompute
    case = tiny_cases["norm_n48_F602"]
    n = int(case["n"])
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.stack([case["rows"], case["cols"]])),
                                  torch.from_numpy(case["vals"]), (n, n)).cuda()
    monkeypatch.setenv("SGC_AMD_DEVICES", "0,0,0,0")
    out, secs = sgc_precompute(torch.from_numpy(case["X"]).cuda(), adj, 2)
    assert secs > 0
    assert np.array_equal(out.cpu().numpy().view(np.uint32), case["Y2"].view(np.uint32))
    assert any(k[0] == "mgpu" for k in adj._sgc_amd_csr[1]._plans if isinstance(k, tuple))


@pytest.mark.slow
def test_mgpu_engine_reddit_shape_hash(shapes_golden):
    """1, 2 and 8 virtual devices at full Reddit shape (602-, 304- and
    76-column blocks: the first two run two column groups per hop inside the
    engine, the last one launch): the reference's X_2 hash each time."""
    from sgc_amd import graphs
    from sgc_amd.multigpu import DeviceSet
    from sgc_amd.propagate import DeviceCSR
    g = shapes_golden["reddit"]
    S = graphs.synthetic_graph("reddit", seed=g["seed"])
    X = torch.from_numpy(graphs.synthetic_features("reddit", g["n"], g["features"],
                                                   seed=g["feature_seed"])).cuda()
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device="cuda")
    for ndev in (1, 2, 8):
        out = torch.empty_like(X)
        DeviceSet.get([0] * ndev).propagate(csr, X, 2, out)
        torch.cuda.synchronize()
        got = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()
        assert got == g["outputs"]["2"]["sha"], ndev


def test_mgpu_handles_survive_reinit(tiny_cases, oracle):
    """Handles are unique for the process: an adjacency attached to an
    engine that was since re-initialised (another device list) is detached
    by its finalizer without touching the adjacency attached to the new
    engine under the same ordinal."""
    import gc
    from sgc_amd.multigpu import DeviceSet
    a = tiny_cases["norm_n48_F130"]
    b = tiny_cases["norm_n48_F65"]
    csr_a = _csr(a, oracle)
    DeviceSet.get([0, 0]).propagate(csr_a, torch.from_numpy(a["X"]).cuda(), 2,
                                    torch.empty(a["X"].shape, device="cuda"))
    csr_b = _csr(b, oracle)
    ds = DeviceSet.get([0, 0, 0])  # re-init: a's handle is void now
    Xb = torch.from_numpy(b["X"]).cuda()
    ds.propagate(csr_b, Xb, 2, torch.empty(b["X"].shape, device="cuda"))
    del csr_a
    gc.collect()  # a's finalizer detaches a's (old) handle
    out = torch.full(b["X"].shape, float("nan"), device="cuda")
    ds.propagate(csr_b, Xb, 2, out)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), b["Y2"].view(np.uint32))


# ---------------------------------------------------------------------------
# the exchanges' block copy (sgc_copy_blocks_f32, csrc/exchange.hip)

@pytest.mark.parametrize("lds,ldd,align", [(64, 602, 4), (76, 602, 2), (96, 608, 4),
                                           (33, 101, 1), (512, 512, 4)])
def test_copy_blocks_matches_slicing(lds, ldd, align):
    """One launch lands up to 64 (src_row, src_col, dst_row, dst_col, rows,
    cols) blocks -- the replicated output's unpack: P column blocks of a
    gathered [P*rows, ld] chunk into X_K's columns, ragged last block, empty
    segments -- exactly as the torch slice copies; 16-B / 8-B / 4-B vectors
    by the strides and offsets, segments longer than the grid (grid-stride
    loop); untouched elements stay."""
    from sgc_amd.distributed import _copy_blocks
    rng = np.random.default_rng(lds * 1000 + ldd)
    rows_src, rows_dst = 9000, 5000
    src = torch.from_numpy(rng.standard_normal((rows_src, lds), dtype=np.float32)).to("cuda")
    dst = torch.full((rows_dst, ldd), float("nan"), device="cuda")
    segs, q, c = [], 0, 0
    while c < ldd and q < 60:
        w = int(min(ldd - c, rng.integers(1, lds + 1) // align * align or align))
        w = min(w, lds)
        r = int(rng.integers(0, 1400))
        sr = int(rng.integers(0, rows_src - r + 1))
        dr = int(rng.integers(0, rows_dst - r + 1))
        sc = int(rng.integers(0, (lds - w) // align + 1)) * align
        segs.append((sr, sc, dr, c, r, w))
        c += w
        q += 1
    segs.append((0, 0, 0, 0, 0, 5))  # empty
    want = dst.clone()
    for sr, sc, dr, dc, r, w in segs:
        want[dr:dr + r, dc:dc + w] = src[sr:sr + r, sc:sc + w]
    _copy_blocks(src, dst, segs)
    torch.cuda.synchronize()
    assert torch.equal(torch.nan_to_num(dst, nan=7.0), torch.nan_to_num(want, nan=7.0))
    # whole 64-block chunk in one launch: the P = 64 limit
    full = torch.from_numpy(rng.standard_normal((64 * 300, 8), dtype=np.float32)).to("cuda")
    out = torch.zeros((300, 64 * 8), device="cuda")
    _copy_blocks(full, out, [(qq * 300, 0, 0, qq * 8, 300, 8) for qq in range(64)])
    torch.cuda.synchronize()
    assert torch.equal(out, full.view(64, 300, 8).permute(1, 0, 2).reshape(300, 512))


def test_copy_blocks_rejects_bad_segments():
    """More than 64 segments, a block past the row stride, negative sizes:
    SGCError, nothing launched."""
    import ctypes
    from sgc_amd import _lib
    lib = _lib.load()
    src = torch.zeros((10, 8), device="cuda")
    dst = torch.zeros((10, 8), device="cuda")

    def call(segs):
        arr = (ctypes.c_int64 * (6 * len(segs)))(*[v for sg in segs for v in sg])
        return lib.sgc_copy_blocks_f32(_lib.ptr(src), 8, _lib.ptr(dst), 8, len(segs), arr,
                                       _lib.stream_handle())
    assert call([(0, 0, 0, 0, 1, 1)] * 65) != 0
    assert call([(0, 4, 0, 0, 1, 8)]) != 0
    assert call([(0, 0, 0, 0, -1, 1)]) != 0
    assert call([(0, 0, 0, 0, 10, 8)]) == 0
    torch.cuda.synchronize()


# ---------------------------------------------------------------------------
# sgc_precompute under torchrun, the reddit driver, bench.py self-launch

@pytest.mark.parametrize("partition", ["features", "lines", "rows", "cyclic", "replicate", "auto"])
def test_sgc_precompute_under_torchrun_matches_one_gpu(tmp_path, partition):
    """Two torchrun ranks sharing the GPU (gloo, chosen by the drop-in because
    there are fewer GPUs than ranks) run the unchanged sgc_precompute on the
    reddit driver's synthetic graph: both get the X_K one GPU computes."""
    from drivers.reddit import synthetic_reddit
    from sgc_amd.utils import sgc_precompute
    r = _torchrun(2, ["tests/rank_precompute.py", str(tmp_path), "20000"],
                  {"SGC_AMD_PARTITION": partition}, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = [json.load(open(tmp_path / f"rank{i}.json")) for i in range(2)]
    adj, _, features, _, _, _, _ = synthetic_reddit(20000)
    one, _ = sgc_precompute(features, adj, 2)
    want = hashlib.sha256(one.cpu().numpy().tobytes()).hexdigest()
    for rec in recs:
        assert rec["world"] == 2 and rec["backend"] == "gloo" and rec["repeat_equal"]
        assert rec["sha"] == want
        assert rec["propagations"] == [1, 1, 1], rec  # no trials in the first call
        if partition in ("features", "lines"):  # replicated X_K by IPC pulls
            assert rec["exchange"] == ["ipc"], rec


@pytest.mark.parametrize("world", [2, 4, 8])
def test_auto_first_call_one_partition_ranks_sharing_gpu(tmp_path, world):
    """VERDICT r05 item 2 on the GPU: `world` torchrun ranks sharing this GPU
    run the unchanged sgc_precompute with the default "auto" partition (the
    minimum-work gate off, so the rule splits at world >= 3): every call,
    the first included, runs exactly one propagation, and every rank's X_K
    is one GPU's; the replicated output of a split goes through the IPC
    window (peers' blocks pulled into X_K, ranks in different processes)."""
    from drivers.reddit import synthetic_reddit
    from sgc_amd.multigpu import rule_choice
    from sgc_amd.utils import sgc_precompute
    n = 20000
    r = _torchrun(world, ["tests/rank_precompute.py", str(tmp_path), str(n)],
                  {"SGC_AMD_AUTO_MIN_WORK": "0"}, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = [json.load(open(tmp_path / f"rank{i}.json")) for i in range(world)]
    adj, _, features, _, _, _, _ = synthetic_reddit(n)
    one, _ = sgc_precompute(features, adj, 2)
    want = hashlib.sha256(one.cpu().numpy().tobytes()).hexdigest()
    chosen = rule_choice(world, n, adj._sgc_amd_csr[1].nnz, features.shape[1], 2) \
        if world > 2 else "replicate"
    for rec in recs:
        assert rec["world"] == world and rec["sha"] == want and rec["repeat_equal"], rec
        assert rec["propagations"] == [1, 1, 1], rec
        assert rec["auto"]["chosen"] == chosen and rec["auto"]["how"] == "rule", rec
        if chosen != "replicate":
            assert rec["exchange"] == ["ipc"], rec


def test_rccl_exchange_paths_world1():
    """The RCCL calls of the feature and line partitions on this one-GPU box
    (tests/rank_rccl_world1.py): a one-rank nccl group with the propagators'
    one-rank shortcuts turned off (force_collectives), so the in-place async
    all-gathers of the last hop's row chunks, their waits on the compute
    stream, the block-copy unpack and the line partition's tail-stream gather
    pattern all run through RCCL; X_K equals one GPU's bit for bit.  (RCCL
    refuses two ranks on one GPU, so this is as far as RCCL runs here.)"""
    r = _torchrun(1, ["tests/rank_rccl_world1.py", "20000"], timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _last_json(r.stdout)
    assert rec["backend"] == "nccl" and rec["world"] == 1, rec
    assert rec["features_replicated_equal"] and rec["lines_replicated_equal"], rec
    assert rec["lines_sharded_equal"] and rec["tail_stream_pattern_ok"], rec
    assert rec["schedules_equal"], rec  # 1:3:3:1 chunks, one / two streams, hub rows early
    # the IPC window at world 1 (force_ipc): handle, flags, waits, pulls
    assert rec["ipc_features_equal"] and rec["ipc_lines_equal"], rec
    assert rec["ipc_scaled_calls_exact"], rec


def test_reddit_driver_runs_under_torchrun():
    """drivers/reddit.py (the reference's reddit.py flow) unchanged under
    torchrun: every rank precomputes through the partitioned path and trains."""
    r = _torchrun(2, ["drivers/reddit.py", "--synthetic", "20000"], timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.count("Total Time:") == 2


def test_bench_self_launch_two_ranks():
    """`bench.py --gpus 2` without torchrun's environment starts its own two
    ranks (gloo: they share this GPU) and prints rank 0's line."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--dist-backend", "gloo", "--shape",
           "pubmed", "--steps", "2", "--warmup", "1", "--sharded-steps", "1"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _last_json(r.stdout)
    assert rec["n_gpus"] == 2 and rec["value"] > 0 and rec["steps"] == 2
    # N > 1 times the same public call as N = 1 (replicated X_K) ...
    assert rec["config"]["output"] == "replicated" and "sgc_precompute" in rec["timed_call"]
    # ... with the roofline's kernel named by the library and a stated basis
    roof = rec["roofline"]
    assert roof["kernel"].startswith("spmm_") and roof["frac"] > 0
    assert roof["compulsory_frac"] == roof["frac"] and "compulsory" in roof["achieved_basis"]
    assert rec["first_call_seconds"] > 0
    # the sharded partitioned path beside it, partition timed on the node
    assert rec["sharded_output"]["value"] > 0
    assert "auto-selected" in rec["sharded_output"]["parallelism"]


# ---------------------------------------------------------------------------
# P = 8 at full size (gloo, 8 ranks on this GPU)

@pytest.fixture(scope="module")
def dist_cache(tmp_path_factory):
    return str(tmp_path_factory.mktemp("dist_check"))


@pytest.mark.slow
@pytest.mark.timeout(900)
@pytest.mark.parametrize("shape,partition,extra", [
    ("reddit", "rows", []),
    ("reddit", "rows", ["--row-chunks", "4"]),
    ("reddit", "cyclic", ["--groups", "3"]),
    ("reddit", "features", ["--also-replicated"]),
    ("reddit", "lines", ["--also-replicated"]),
    ("reddit", "tiles", ["--col-blocks", "2"]),
    ("rmat", "rows", []),
    ("rmat", "lines", [])])  # the P = 8 layout at F = 256: one 32-float line per rank
def test_p8_partition_full_size_bit_exact(dist_cache, shape, partition, extra):
    r = _torchrun(8, ["scripts/dist_check.py", "--shape", shape, "--partition", partition,
                      "--cache", dist_cache, *extra], timeout=840)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _last_json(r.stdout)
    assert rec["world"] == 8 and rec["bit_exact_vs_reference_hash"], rec
    if "--also-replicated" in extra:  # every rank's full X_K: IPC pulls and the collective
        assert rec["replicated_exchange"] == ["ipc"], rec
        assert all(rec["replicated"].values()), rec


@pytest.mark.slow
@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,extra", [
    (2, ["--exchange", "pairwise"]),
    (4, ["--exchange", "pairwise", "--pieces", "3"]),
    (2, ["--exchange", "alltoall"])])
def test_feature_partition_exchange_full_size_bit_exact(dist_cache, world, extra):
    """The feature partition's sharded exchange at world 2 / 4 (pairwise P2P
    overlapped with the last hop, the default at world 2; or the all-to-all), full
    Reddit shape: X_K assembled from the ranks' row blocks equals the
    reference's hash."""
    r = _torchrun(world, ["scripts/dist_check.py", "--shape", "reddit", "--partition", "features",
                          "--cache", dist_cache, *extra], timeout=540)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _last_json(r.stdout)
    assert rec["world"] == world and rec["bit_exact_vs_reference_hash"], rec
