"""HIP path parity: sgc_amd on the GPU vs the reference's golden vectors.

Bit-exact (fp32 bit patterns equal) for the propagation; tolerance for the
MFMA classifier (rtol=atol=1e-5 relative to max|ref|, north_star's bar for fp32).
All calls go through libsgc_amd.so; nothing here may fall back to torch ops
for the arithmetic under test.
"""
import functools
import hashlib

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def bits_equal(a, b):
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


def coo_cuda(c):
    n = int(c["n"])
    idx = torch.from_numpy(np.stack([c["rows"], c["cols"]]).astype(np.int64))
    return torch.sparse_coo_tensor(idx, torch.from_numpy(c["vals"]), (n, n)).to(DEV)


@pytest.fixture(scope="module", autouse=True)
def _native_loaded():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    from sgc_amd import _lib
    _lib.load()  # fails loudly if libsgc_amd.so is missing


def test_tiny_cases_sgc_precompute_bit_exact(tiny_cases):
    from sgc_amd.utils import sgc_precompute
    for name, c in tiny_cases.items():
        adj = coo_cuda(c)
        X = torch.from_numpy(c["X"]).to(DEV)
        for key in sorted(k for k in c if k.startswith("Y")):
            K = int(key[1:])
            out, secs = sgc_precompute(X, adj, K)
            if K == 0:
                assert out is X  # reference returns the same object
                continue
            assert secs > 0
            assert bits_equal(out.cpu().numpy(), c[key]), (name, K)


@pytest.mark.parametrize("rows_per_wave", [0, 1, 2, 4])
@pytest.mark.parametrize("hub_chunk", [0, 32, 64])
@pytest.mark.parametrize("threshold,hub", [(0, 0), (1, 7), (7, 7), (63, 500), (0, 10**9),
                                           (10**9, 10**9), (2048, 4096)])
def test_heavy_split_schedule_never_changes_bits(tiny_cases, threshold, hub, hub_chunk,
                                                 rows_per_wave):
    """Every row a hub (0, 0), every row heavy (0, inf) .. no heavy rows, hub
    kernel on 32- or 64-feature chunks, light rows one / two / four per wave
    (spmm_csr_kernel / spmm_rows_kernel): same bits."""
    from sgc_amd import _lib
    lib = _lib.load()
    _lib.check(lib.sgc_set_tuning(b"hub_chunk", hub_chunk), "set_tuning")
    _lib.check(lib.sgc_set_tuning(b"rows_per_wave", rows_per_wave), "set_tuning")
    try:
        _schedule_cases(tiny_cases, threshold, hub)
    finally:
        lib.sgc_set_tuning(b"hub_chunk", 0)
        lib.sgc_set_tuning(b"rows_per_wave", 0)


@pytest.mark.parametrize("F", [128, 304, 300, 152])
def test_wide_launch_kernel_choice_bit_exact(oracle, F):
    """Launches of >= 65,536 rows: at F = 128 and F > 256 with 16-B lanes the
    multi-row kernel runs (128-float slices), at 152 the one-row kernel; both
    in the engine's padded buffers (the feature partition's P = 2 / P = 4
    blocks) and in a caller's unpadded tensor: the oracle's bits."""
    from sgc_amd import graphs
    from sgc_amd.propagate import SPMM_X_PADDED, SPMM_Y_PADDED, DeviceCSR, spmm
    n = 70000
    S = graphs.synthetic_graph("pubmed", seed=5, n=n, edges=350000)
    X = np.random.default_rng(F).standard_normal((n, F)).astype(np.float32)
    want = oracle.spmm_csr(S.row_ptr, S.col_idx, S.val, X, 0, n)
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device=DEV)
    ld = (F + 31) // 32 * 32
    Xp = torch.zeros((n, ld), device=DEV)
    Xp[:, :F] = torch.from_numpy(X)
    Yp = torch.full((n, ld), float("nan"), device=DEV)
    for th, hub in ((None, None), (16, 200), (10**9, 10**9)):
        kw = {} if th is None else {"threshold": th, "hub_threshold": hub}
        spmm(csr, Xp[:, :F], 0, n, out=Yp[:, :F], flags=SPMM_X_PADDED | SPMM_Y_PADDED, **kw)
        y = spmm(csr, Xp[:, :F].contiguous(), 0, n, **kw)
        torch.cuda.synchronize()
        assert bits_equal(Yp[:, :F].cpu().numpy(), want), (F, th)
        assert bits_equal(y.cpu().numpy(), want), (F, th)


def _schedule_cases(tiny_cases, threshold, hub):
    from sgc_amd.propagate import DeviceCSR, propagate
    for name in ("hub1000_F65", "hub1000_F130", "norm_n48_F602", "norm_n48_F130",
                 "norm_n48_F3", "raw_sorted_dups_F66", "raw_unsorted_dups_F7", "special_values_F11",
                 "isolated_F17"):
        c = tiny_cases[name]
        csr = DeviceCSR.from_torch(coo_cuda(c))
        X = torch.from_numpy(c["X"]).to(DEV)
        for key in sorted(k for k in c if k.startswith("Y") and k != "Y0"):
            out = propagate(csr, X, int(key[1:]), threshold=threshold, hub_threshold=hub)
            torch.cuda.synchronize()
            assert bits_equal(out.cpu().numpy(), c[key]), (name, key, threshold, hub)


def test_no_plan_path(tiny_cases):
    from sgc_amd.propagate import DeviceCSR, propagate
    c = tiny_cases["hub1000_F65"]
    csr = DeviceCSR.from_torch(coo_cuda(c))
    out = propagate(csr, torch.from_numpy(c["X"]).to(DEV), 2, use_plan=False)
    assert bits_equal(out.cpu().numpy(), c["Y2"])


@pytest.mark.parametrize("native", [False, True])
@pytest.mark.parametrize("ld_extra", [0, 38, 3])
@pytest.mark.parametrize("name", ["norm_n48_F602", "norm_n48_F65", "norm_n48_F130"])
def test_propagate_layouts_and_native_loop(tiny_cases, native, ld_extra, name):
    """Python hop loop and the C ABI loop (sgc_propagate_f32), with inputs
    needing the 128-B re-layout (ld F / F+3) and not (ld F+38 when that is a
    multiple of 32), at F = 602 / 65 / 130 (pad columns up to a multiple of 4
    computed inside the engine's buffers, never in the caller's)."""
    from sgc_amd.propagate import DeviceCSR, propagate
    c = tiny_cases[name]
    F = c["X"].shape[1]
    csr = DeviceCSR.from_torch(coo_cuda(c))
    X = torch.from_numpy(c["X"]).to(DEV)
    buf = torch.full((X.shape[0], F + ld_extra), float("nan"), device=DEV)
    buf[:, :F] = X
    for K in (0, 1, 2, 3):
        out = torch.full((X.shape[0], F + 5), float("nan"), device=DEV)
        got = propagate(csr, buf[:, :F], K, out=out[:, :F], native_loop=native)
        torch.cuda.synchronize()
        assert bits_equal(got.cpu().numpy(), c[f"Y{K}"]), (K, native, ld_extra)
        assert torch.isnan(out[:, F:]).all()  # nothing written past F in the caller's rows


def test_row_slices_and_strides(tiny_cases):
    """Row-range SpMM (the multi-GPU shard kernel) + padded strides."""
    from sgc_amd.propagate import DeviceCSR, spmm
    c = tiny_cases["norm_n48_F602"]
    csr = DeviceCSR.from_torch(coo_cuda(c))
    X = torch.from_numpy(c["X"]).to(DEV)
    Xpad = torch.zeros((X.shape[0], 640), device=DEV)
    Xpad[:, :602] = X
    full = c["Y1"]
    for lo, hi in ((0, 5), (5, 31), (31, 48), (10, 10)):
        for Xin in (X, Xpad[:, :602]):
            out = torch.full((hi - lo, 700), float("nan"), device=DEV)
            spmm(csr, Xin, lo, hi, out=out[:, :602], threshold=3, hub_threshold=5)
            torch.cuda.synchronize()
            o = out.cpu().numpy()
            assert bits_equal(o[:, :602], full[lo:hi])
            assert np.isnan(o[:, 602:]).all()  # no writes past F


def test_ingest_status_and_csr(tiny_cases, oracle):
    from sgc_amd.propagate import (STATUS_COLS_ASCENDING, STATUS_ROWS_SORTED, DeviceCSR)
    c = tiny_cases["norm_n48_F64"]
    csr = DeviceCSR.from_torch(coo_cuda(c))
    assert csr.status & STATUS_ROWS_SORTED and csr.status & STATUS_COLS_ASCENDING
    c = tiny_cases["raw_unsorted_dups_F7"]
    csr = DeviceCSR.from_torch(coo_cuda(c))
    assert not csr.status & STATUS_ROWS_SORTED
    n = int(c["n"])
    rp, ci, va = oracle.coo_to_csr(n, n, c["rows"], c["cols"], c["vals"])
    assert np.array_equal(csr.row_ptr.cpu().numpy(), rp)
    assert np.array_equal(csr.col_idx.cpu().numpy(), ci)
    assert bits_equal(csr.val.cpu().numpy(), va)
    c = tiny_cases["raw_sorted_dups_F66"]
    csr = DeviceCSR.from_torch(coo_cuda(c))
    assert csr.status & STATUS_ROWS_SORTED and not csr.status & STATUS_COLS_ASCENDING


def test_csr_layout_input(tiny_cases):
    from sgc_amd.utils import sgc_precompute
    c = tiny_cases["norm_n48_F65"]
    adj = coo_cuda(c).cpu().to_sparse_csr().to(DEV)
    out, _ = sgc_precompute(torch.from_numpy(c["X"]).to(DEV), adj, 2)
    assert bits_equal(out.cpu().numpy(), c["Y2"])


def test_errors_are_loud(tiny_cases):
    from sgc_amd._lib import SGCError
    from sgc_amd.utils import sgc_precompute
    c = tiny_cases["norm_n48_F3"]
    adj = coo_cuda(c)
    with pytest.raises(RuntimeError):  # CPU features with a GPU adjacency
        sgc_precompute(torch.from_numpy(c["X"]), adj, 2)
    with pytest.raises(RuntimeError):  # shape mismatch
        sgc_precompute(torch.zeros((5, 3), device=DEV), adj, 1)
    bad = torch.sparse_coo_tensor(torch.tensor([[0, 1], [1, 7]]), torch.tensor([1.0, 2.0]), (3, 3),
                                  check_invariants=False).to(DEV)
    with pytest.raises(SGCError):
        sgc_precompute(torch.zeros((3, 4), device=DEV), bad, 1)


def test_cache_invalidation_on_inplace_update(tiny_cases):
    from sgc_amd.utils import sgc_precompute
    c = tiny_cases["norm_n48_F65"]
    adj = coo_cuda(c)
    X = torch.from_numpy(c["X"]).to(DEV)
    out1, _ = sgc_precompute(X, adj, 1)
    assert bits_equal(out1.cpu().numpy(), c["Y1"])
    adj._values().mul_(2.0)  # bumps _version -> CSR rebuilt
    out2, _ = sgc_precompute(X, adj, 1)
    assert not bits_equal(out2.cpu().numpy(), c["Y1"])


@pytest.mark.parametrize("shape", ["cora", "pubmed"])
def test_shape_hashes(shape, shapes_golden, shape_rows):
    from sgc_amd import graphs
    from sgc_amd.propagate import DeviceCSR, propagate
    g = shapes_golden[shape]
    S = graphs.synthetic_graph(shape, seed=g["seed"])
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val)
    X = graphs.synthetic_features(shape, g["n"], g["features"], seed=g["feature_seed"])
    Xd = torch.from_numpy(X).to(DEV)
    for K, rec in g["outputs"].items():
        Y = propagate(csr, Xd, int(K)).cpu().numpy()
        assert bits_equal(Y[shape_rows[f"{shape}_rows"]], shape_rows[f"{shape}_K{K}"]), (shape, K)
        assert sha(Y) == rec["sha"], (shape, K)


@functools.lru_cache(maxsize=1)
def _big_graph(shape, seed):
    """The seeded BASELINE-shape graph, generated once for the tests that
    follow each other on it (the RMAT shape takes a minute on the host)."""
    from sgc_amd import graphs
    return graphs.synthetic_graph(shape, seed=seed)


def device_sha(Y):
    """SHA-256 of a device tensor's bytes, copied to the host in 256 MB
    pieces (the same digest as sha(Y.cpu().numpy()))."""
    h = hashlib.sha256()
    rows = max(1, (256 << 20) // max(1, 4 * Y.shape[1]))
    for r in range(0, Y.shape[0], rows):
        h.update(np.ascontiguousarray(Y[r:r + rows].cpu().numpy()).tobytes())
    return h.hexdigest()


def _public_call_hashes(shape, K, g, calls):
    """The call bench.py times, as bench.py makes it: the public
    sgc_precompute(X, adj, K) on a torch COO adjacency moved to the GPU
    (device ingest + plan + recording on the first call, the recorded launch
    list replayed on later ones).  `calls` lists, per call, whether it gets
    the same X tensor ("same") or a fresh copy of it ("new"); every call's
    result is a new X_K tensor.  Returns each call's output hash."""
    from sgc_amd import graphs
    from sgc_amd.utils import sgc_precompute
    S = _big_graph(shape, g["seed"])
    X = graphs.synthetic_features(shape, g["n"], g["features"], seed=g["feature_seed"])
    rows, cols, vals = S.coo()
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.stack([rows, cols])),
                                  torch.from_numpy(vals), (S.n, S.n)).to(DEV)
    del rows, cols, vals
    X0 = torch.from_numpy(X).to(DEV)
    del X
    hashes, outs = [], []
    for kind in calls:
        Xc = X0 if kind == "same" else X0.clone()
        out, secs = sgc_precompute(Xc, adj, K)
        assert secs > 0 and out.shape == X0.shape
        hashes.append(device_sha(out))
        outs.append(out.data_ptr())
        del out, Xc
    assert getattr(adj, "_sgc_amd_csr", None) is not None  # the CSR was cached
    del X0, adj
    torch.cuda.empty_cache()
    return hashes


@pytest.mark.slow
def test_public_call_reddit_shape_hash_replay(shapes_golden):
    """the exact call bench.py times at the benched size
    -- sgc_precompute(features, adj, 2) on the Reddit-shape torch COO (reference
    reddit.py:43 -> utils.py:92-97) -- hashed on the first call (device ingest,
    plan, launch-list recording), on a replay with the same X_0 and on a
    replay with a new X_0 tensor, all against the reference's own hash."""
    g = shapes_golden["reddit"]
    want = g["outputs"]["2"]["sha"]
    hashes = _public_call_hashes("reddit", 2, g, ["same", "same", "new"])
    assert hashes == [want] * 3, hashes


@pytest.mark.slow
def test_reddit_shape_hash(shapes_golden, shape_rows):
    """Full BASELINE size (233k nodes, 23.4M nnz, F=602, K=2): bit-exact hash
    of the whole output against the reference's torch.spmm result."""
    if "reddit" not in shapes_golden:
        pytest.skip("reddit golden not generated")
    from sgc_amd import graphs
    from sgc_amd.propagate import DeviceCSR, propagate
    g = shapes_golden["reddit"]
    S = _big_graph("reddit", g["seed"])
    rows, cols, vals = S.coo()
    assert sha(np.stack([rows, cols])) == g["sha_indices"]
    assert sha(vals) == g["sha_values"]
    X = graphs.synthetic_features("reddit", g["n"], g["features"], seed=g["feature_seed"])
    assert sha(X) == g["sha_X"]
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val)
    Y = propagate(csr, torch.from_numpy(X).to(DEV), 2).cpu().numpy()
    assert bits_equal(Y[shape_rows["reddit_rows"]], shape_rows["reddit_K2"])
    assert sha(Y) == g["outputs"]["2"]["sha"]


@pytest.mark.slow
def test_rmat_shape_hash(shapes_golden, shape_rows):
    """BASELINE config 5 at full size (4,194,304 nodes, 260,194,304 nnz, F=256,
    K=3): bit-exact hash of the whole X_3 against the reference's own
    sgc_precompute (tests/golden/gen_golden.py rmat, run in the build
    container: reference aug_normalized_adjacency + sparse_mx_to_torch_sparse_
    tensor + torch.spmm COO, 308 s on one CPU thread)."""
    if "rmat" not in shapes_golden:
        pytest.skip("rmat golden not generated")
    from sgc_amd import graphs
    from sgc_amd.propagate import DeviceCSR, propagate
    g = shapes_golden["rmat"]
    S = _big_graph("rmat", g["seed"])
    rows, cols, vals = S.coo()
    assert sha(np.stack([rows, cols])) == g["sha_indices"]
    assert sha(vals) == g["sha_values"]
    del rows, cols, vals
    X = graphs.synthetic_features("rmat", g["n"], g["features"], seed=g["feature_seed"])
    assert sha(X) == g["sha_X"]
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val)
    Xd = torch.from_numpy(X)
    del X
    Y = propagate(csr, Xd.to(DEV), 3).cpu().numpy()
    assert bits_equal(Y[shape_rows["rmat_rows"]], shape_rows["rmat_K3"])
    assert sha(Y) == g["outputs"]["3"]["sha"]


@pytest.mark.slow
def test_public_call_rmat_shape_hash_replay(shapes_golden):
    """BASELINE config 5 through the public call as bench.py times it: the
    first call (device ingest of 260 M COO entries, plan, recording) and one
    launch-list replay with a new X_0, hashed against the reference's X_3."""
    g = shapes_golden["rmat"]
    hashes = _public_call_hashes("rmat", 3, g, ["same", "new"])
    assert hashes == [g["outputs"]["3"]["sha"]] * 2, hashes


@pytest.mark.parametrize("F", [64, 130, 192])
@pytest.mark.parametrize("hub_chunk", [32, 64])
@pytest.mark.parametrize("hub_loaders", [15, 7])
def test_long_hub_rows_bit_exact(oracle, F, hub_chunk, hub_loaders):
    """Hub rows of 7,000 / 3,001 / 2,881 nonzeros on the LDS-staged hub kernel:
    several kHubUnroll iterations (2,880 nonzeros each at HC=32), the
    register-ring and column-id parity wrap, and ragged last rounds, on
    128-B aligned rows (HC=32 is what the row partition's narrow feature
    groups use).  Oracle: the CPU restatement of torch.spmm's arithmetic."""
    from sgc_amd import _lib, graphs
    from sgc_amd.propagate import DeviceCSR, propagate
    rng = np.random.default_rng(F + hub_chunk)
    n = 9000
    u = [np.zeros(7000, np.int64), np.full(3001, 1, np.int64), np.full(2881, 2, np.int64)]
    v = [np.arange(1000, 8000), np.arange(3000, 6001), np.arange(5000, 7881)]
    ru, rv = rng.integers(3, n, 20000), rng.integers(3, n, 20000)
    keep = ru != rv
    lo = np.concatenate(u + [np.minimum(ru, rv)[keep]])
    hi = np.concatenate(v + [np.maximum(ru, rv)[keep]])
    key = np.unique(lo * n + hi)
    S = graphs.aug_norm_csr_from_pairs(n, key // n, key % n)
    X = rng.standard_normal((n, F)).astype(np.float32)
    want = oracle.propagate(S.row_ptr, S.col_idx, S.val, X, 2)
    lib = _lib.load()
    _lib.check(lib.sgc_set_tuning(b"hub_chunk", hub_chunk), "set_tuning")
    _lib.check(lib.sgc_set_tuning(b"hub_loaders", hub_loaders), "set_tuning")
    try:
        csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val)
        pl = csr.plan(0, n, 64, 1000, F)
        assert pl.n_hub == 3
        Xd = torch.zeros((n, (F + 31) // 32 * 32), device=DEV)[:, :F]  # 128-B rows
        Xd.copy_(torch.from_numpy(X))
        out = propagate(csr, Xd, 2, threshold=64, hub_threshold=1000)
        torch.cuda.synchronize()
        assert bits_equal(out.cpu().numpy(), want)
    finally:
        lib.sgc_set_tuning(b"hub_chunk", 0)
        lib.sgc_set_tuning(b"hub_loaders", 15)


@pytest.mark.parametrize("heavy_pairs", [1, 5, 13, 17])
@pytest.mark.parametrize("F", [1, 3, 4, 12, 16, 17, 30, 32, 33, 36, 44, 60, 64, 76, 96, 100, 124,
                               152])
def test_narrow_launches_rows_kernel(oracle, F, heavy_pairs):
    """Feature widths below a slice (the feature partition's column blocks,
    the row partition's narrow groups): spmm_rows_kernel packs 64 // (F/4)
    rows into a wave.  Heavy rows (threshold 40) and hub rows (500) on the
    same launch, heavy rows two nonzeros per load (heavy_pairs 1) or four:
    up to 32 floats row_quads_pipe with 2- or 1-float lanes (5), at 33..64
    floats the transposed quads (13: row_quadsT_pipe, 16-B lanes); X in
    128-B rows so hop 1 also takes 16-B lanes."""
    from sgc_amd import _lib, graphs
    from sgc_amd.propagate import DeviceCSR, propagate
    lib = _lib.load()
    prev = lib.sgc_get_tuning(b"heavy_pairs")
    _lib.check(lib.sgc_set_tuning(b"heavy_pairs", heavy_pairs), "set_tuning")
    try:
        _narrow_case(oracle, F)
    finally:
        lib.sgc_set_tuning(b"heavy_pairs", prev)


def _narrow_case(oracle, F):
    from sgc_amd import graphs
    from sgc_amd.propagate import DeviceCSR, propagate
    rng = np.random.default_rng(F)
    n = 3000
    lo = np.concatenate([np.zeros(900, np.int64), np.full(300, 7, np.int64),
                         rng.integers(0, n, 15000)])
    hi = np.concatenate([np.arange(100, 1000), np.arange(1000, 1300), rng.integers(0, n, 15000)])
    keep = lo != hi
    a, b = np.minimum(lo, hi)[keep], np.maximum(lo, hi)[keep]
    key = np.unique(a * n + b)
    S = graphs.aug_norm_csr_from_pairs(n, key // n, key % n)
    X = rng.standard_normal((n, F)).astype(np.float32)
    want = oracle.propagate(S.row_ptr, S.col_idx, S.val, X, 2)
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val)
    Xd = torch.zeros((n, (F + 31) // 32 * 32), device=DEV)[:, :F]
    Xd.copy_(torch.from_numpy(X))
    for th, hub in ((40, 500), (10**9, 10**9)):
        out = propagate(csr, Xd, 2, threshold=th, hub_threshold=hub)
        torch.cuda.synchronize()
        assert bits_equal(out.cpu().numpy(), want), (F, th, hub)


def _column_split(S, bounds):
    """S's nonzeros split by column range [bounds[g], bounds[g+1]): one CSR per
    range over the same rows (each row's runs stay in CSR order)."""
    rp, ci, va = (np.asarray(S.row_ptr, np.int64), np.asarray(S.col_idx),
                  np.asarray(S.val))
    n = rp.size - 1
    row = np.repeat(np.arange(n), np.diff(rp))
    grp = np.searchsorted(np.asarray(bounds), ci, side="right") - 1
    out = []
    for g in range(len(bounds) - 1):
        m = grp == g
        sub_rp = np.zeros(n + 1, np.int64)
        np.cumsum(np.bincount(row[m], minlength=n), out=sub_rp[1:])
        out.append((sub_rp.astype(np.int32), ci[m], va[m]))
    return out


@pytest.mark.parametrize("F", [602, 256, 130, 64, 36, 30, 12])
@pytest.mark.parametrize("rows_per_wave", [0, 1, 2])
@pytest.mark.parametrize("th,hub", [(40, 500), (10**9, 10**9)])
def test_accumulate_column_block_passes(oracle, F, rows_per_wave, th, hub):
    """SGC_SPMM_ACCUMULATE: one plain pass over column block 0 of S, then
    accumulate passes over blocks 1, 2, ... (the cyclic multi-GPU pipeline's
    hop) equal one pass over S bit for bit -- light, heavy and hub rows, both
    light kernels, padded 128-B-row buffers (F = 602) and unpadded ones,
    full and partial row ranges.  The output starts as NaN: the plain first
    pass must write every row (zeros where block 0 has no nonzeros), and
    accumulate passes must leave rows without nonzeros in their block as
    they are."""
    from sgc_amd import _lib, graphs
    from sgc_amd.propagate import SPMM_ACCUMULATE, SPMM_X_PADDED, SPMM_Y_PADDED, DeviceCSR, spmm
    rng = np.random.default_rng(F + rows_per_wave)
    n = 3000
    lo = np.concatenate([np.zeros(900, np.int64), np.full(300, 7, np.int64),
                         rng.integers(0, n, 15000)])
    hi = np.concatenate([np.arange(100, 1000), np.arange(1000, 1300), rng.integers(0, n, 15000)])
    keep = lo != hi
    a, b = np.minimum(lo, hi)[keep], np.maximum(lo, hi)[keep]
    key = np.unique(a * n + b)
    S = graphs.aug_norm_csr_from_pairs(n, key // n, key % n)
    X = rng.standard_normal((n, F)).astype(np.float32)
    want = oracle.spmm_csr(S.row_ptr, S.col_idx, S.val, X, 0, n)
    ld = (F + 31) // 32 * 32
    padded = F % 4 != 0 or F == 602
    Xd = torch.zeros((n, ld if padded else F), device=DEV)[:, :F]
    Xd.copy_(torch.from_numpy(X))
    pad_flags = (SPMM_X_PADDED | SPMM_Y_PADDED) if padded else 0
    lib = _lib.load()
    _lib.check(lib.sgc_set_tuning(b"rows_per_wave", rows_per_wave), "set_tuning")
    try:
        for bounds in ([0, 700, 1100, 1600, n], [0, 5, n], [0, n]):
            subs = [DeviceCSR.from_host_arrays(*t, n_cols=n) for t in _column_split(S, bounds)]
            for r0, r1 in ((0, n), (5, 2300)):
                out = torch.full((r1 - r0, ld if padded else F), float("nan"), device=DEV)[:, :F]
                for g, csr in enumerate(subs):
                    spmm(csr, Xd, r0, r1, out=out, threshold=th, hub_threshold=hub,
                         flags=pad_flags | (SPMM_ACCUMULATE if g else 0))
                torch.cuda.synchronize()
                assert bits_equal(out.cpu().numpy(), want[r0:r1]), (bounds, r0, r1)
    finally:
        lib.sgc_set_tuning(b"rows_per_wave", 0)


@pytest.mark.parametrize("fuse", [0, 1])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_hub_stream_modes_bit_exact(tiny_cases, oracle, mode, fuse):
    """Hub kernel beside the light kernel (side stream, fork/join), in line
    before it (SGC_SPMM_HUB_SERIAL / hub_stream=2) or per the plan's longest
    hub row (default); serial hub rows inside the multi-row kernel's launch
    (hub_fuse 1: F = 130 in 128-B rows) or as their own launch: the same
    bits."""
    from sgc_amd import _lib
    from sgc_amd.propagate import DeviceCSR, HUB_SERIAL_MAX_DEGREE, propagate
    lib = _lib.load()
    _lib.check(lib.sgc_set_tuning(b"hub_stream", mode), "set_tuning")
    _lib.check(lib.sgc_set_tuning(b"hub_fuse", fuse), "set_tuning")
    try:
        for name in ("hub1000_F130", "hub1000_F65", "norm_n48_F602"):
            c = tiny_cases[name]
            n = int(c["n"])
            rp, ci, va = oracle.coo_to_csr(n, n, c["rows"], c["cols"], c["vals"])
            csr = DeviceCSR.from_host_arrays(rp, ci, va)
            pl = csr.plan(0, n, 7, 7, c["X"].shape[1])
            if name.startswith("hub"):
                assert 0 < pl.max_hub_degree <= HUB_SERIAL_MAX_DEGREE
            out = propagate(csr, torch.from_numpy(c["X"]).to(DEV), 2, threshold=7, hub_threshold=7)
            torch.cuda.synchronize()
            assert bits_equal(out.cpu().numpy(), c["Y2"]), (name, mode, fuse)
    finally:
        lib.sgc_set_tuning(b"hub_stream", 0)
        lib.sgc_set_tuning(b"hub_fuse", 1)


def test_accumulate_requires_out():
    from sgc_amd.propagate import SPMM_ACCUMULATE, DeviceCSR, spmm
    csr = DeviceCSR.from_host_arrays(np.array([0, 1], np.int32), np.array([0], np.int32),
                                     np.ones(1, np.float32))
    with pytest.raises(ValueError, match="ACCUMULATE"):
        spmm(csr, torch.ones(1, 4, device=DEV), flags=SPMM_ACCUMULATE)


def test_empty_csr_writes_zeros():
    """A CSR without a single nonzero (an empty shard: torch's empty col/val
    tensors have no storage) writes +0.0 rows, like torch.spmm."""
    from sgc_amd.propagate import DeviceCSR, spmm
    csr = DeviceCSR.from_host_arrays(np.zeros(6, np.int32), np.zeros(0, np.int32),
                                     np.zeros(0, np.float32), n_cols=7)
    X = torch.randn(7, 65, device=DEV)
    out = torch.full((5, 65), float("nan"), device=DEV)
    spmm(csr, X, out=out)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    assert np.array_equal(o.view(np.uint32), np.zeros_like(o).view(np.uint32))


def test_fused_xent_rejects_bad_labels():
    from sgc_amd.propagate import linear_xent
    X = torch.randn(10, 8, device=DEV)
    W = torch.randn(3, 8, device=DEV)
    b = torch.zeros(3, device=DEV)
    for bad in (3, -1, -100):
        y = torch.zeros(10, dtype=torch.int64, device=DEV)
        y[4] = bad
        with pytest.raises(ValueError):
            linear_xent(X, W, b, y)


@pytest.mark.parametrize("fuse", [0, 1])
def test_kernel_timing_hooks(tiny_cases, fuse):
    """sgc_timing_*: one (light, hub) pair per SpMM launch, hub None without
    hubs -- and None as well when the (serial) hub rows ran inside the light
    launch (hub_fuse 1: the light kernel's time covers them)."""
    from sgc_amd import _lib
    from sgc_amd.propagate import (DeviceCSR, collect_kernel_timing, kernel_timing,
                                   propagate)
    lib = _lib.load()
    c = tiny_cases["hub1000_F130"]
    csr = DeviceCSR.from_torch(coo_cuda(c))
    X = torch.from_numpy(c["X"]).to(DEV)
    collect_kernel_timing()
    _lib.check(lib.sgc_set_tuning(b"hub_fuse", fuse), "set_tuning")
    kernel_timing(True)
    try:
        out = propagate(csr, X, 2, threshold=3, hub_threshold=5)
        propagate(csr, X, 1, threshold=10**9, hub_threshold=10**9)
    finally:
        kernel_timing(False)
        lib.sgc_set_tuning(b"hub_fuse", 1)
    light, hub = collect_kernel_timing()
    assert len(light) == 3 and all(t > 0 for t in light)
    if fuse:
        # hop 2 (X_1 in the engine's 16-B-lane rows) fused; hop 1 reads the
        # caller's X_0 (F = 130: 8-B lanes), which the fused launch cannot
        # take, so its hub rows run just before the light launch
        assert hub[0] > 0 and hub[1] is None and hub[2] is None
    else:
        assert hub[0] > 0 and hub[1] > 0 and hub[2] is None
    assert bits_equal(out.cpu().numpy(), c["Y2"])
    assert collect_kernel_timing() == ([], [])


def test_hub_fusion_hop1_with_16B_rows(tiny_cases, oracle):
    """Hop 1 fuses its hub rows too when the caller's X_0 gives 16-B lanes
    (F % 4 == 0, 16-B aligned rows -- Pubmed's F = 500): no hub launch on any
    hop, bit-exact against the oracle."""
    from sgc_amd import _lib
    from sgc_amd.propagate import DeviceCSR, collect_kernel_timing, kernel_timing, propagate
    lib = _lib.load()
    c = tiny_cases["hub1000_F130"]
    n = int(c["n"])
    X0 = np.ascontiguousarray(c["X"][:, :128])
    rp, ci, va = oracle.coo_to_csr(n, n, c["rows"], c["cols"], c["vals"])
    want = oracle.propagate(rp, ci, va, X0, 2)
    csr = DeviceCSR.from_torch(coo_cuda(c))
    X = torch.from_numpy(X0).to(DEV)
    collect_kernel_timing()
    _lib.check(lib.sgc_set_tuning(b"hub_fuse", 1), "set_tuning")
    kernel_timing(True)
    try:
        out = propagate(csr, X, 2, threshold=3, hub_threshold=5)
    finally:
        kernel_timing(False)
    light, hub = collect_kernel_timing()
    assert len(light) == 2 and hub == [None, None], hub
    assert bits_equal(out.cpu().numpy(), want)


@pytest.mark.parametrize("M,K,C", [(1, 3, 1), (140, 1433, 7), (333, 602, 41), (1000, 500, 3),
                                   (77, 64, 64), (50, 130, 100), (2048, 602, 41), (8192, 602, 41),
                                   (5000, 1433, 7), (4096, 3703, 6), (6000, 500, 3)])
def test_linear_mfma_vs_torch_fp32(M, K, C):
    from sgc_amd.propagate import linear
    g = torch.Generator().manual_seed(M * 7 + K)
    X = torch.randn((M, K), generator=g)
    W = torch.randn((C, K), generator=g) * 0.05
    b = torch.randn(C, generator=g)
    ref = torch.nn.functional.linear(X.double(), W.double(), b.double()).float()
    Y = linear(X.to(DEV), W.to(DEV), b.to(DEV)).cpu()
    tol = 1e-5 * max(1.0, ref.abs().max().item())
    torch.testing.assert_close(Y, ref, rtol=1e-5, atol=tol)
    Yn = linear(X.to(DEV), W.to(DEV), None).cpu()
    torch.testing.assert_close(Yn, ref - b, rtol=1e-5, atol=tol)


@pytest.mark.parametrize("tile_buffers", [1, 2])
@pytest.mark.parametrize("M,K,C,ld_extra", [(129, 602, 41, 6), (300, 33, 17, 0), (257, 31, 3, 1),
                                            (128, 64, 64, 32), (1, 1, 1, 3), (500, 602, 70, 2)])
def test_linear_tile_edges(tile_buffers, M, K, C, ld_extra):
    """The classifier tile's buffer loads (gemm_tile.h): rows past M, classes
    past C and the k >= K tail of the last chunk read as zeros -- X's columns
    past K hold infinities here, so an unmasked tail would give NaN -- with one
    or two LDS images; forward and the fused step's logits."""
    from sgc_amd import _lib
    from sgc_amd.propagate import linear, linear_xent
    lib = _lib.load()
    g = torch.Generator().manual_seed(M + K + C)
    Xf = torch.full((M, K + ld_extra), float("inf"))
    Xf[:, :K] = torch.randn((M, K), generator=g)
    W = torch.randn((C, K), generator=g) * 0.05
    b = torch.randn(C, generator=g)
    y = torch.randint(0, C, (M,), generator=g)
    ref = torch.nn.functional.linear(Xf[:, :K].double(), W.double(), b.double())
    tol = 1e-5 * max(1.0, ref.abs().max().item())
    _lib.check(lib.sgc_set_tuning(b"tile_buffers", tile_buffers), "set_tuning")
    try:
        Xd = Xf.to(DEV)[:, :K]
        Y = linear(Xd, W.to(DEV), b.to(DEV)).cpu().double()
        torch.testing.assert_close(Y, ref, rtol=1e-5, atol=tol)
        if C <= 64:
            _, _, _, logits = linear_xent(Xd, W.to(DEV), b.to(DEV), y.to(DEV), want_logits=True)
            torch.testing.assert_close(logits.cpu().double(), ref, rtol=1e-5, atol=tol)
    finally:
        lib.sgc_set_tuning(b"tile_buffers", 1)


@pytest.mark.parametrize("M,K,C,ld_extra", [(129, 602, 41, 6), (300, 33, 17, 1), (257, 31, 3, 1),
                                            (128, 64, 64, 32), (1, 1, 1, 1), (500, 576, 70, 2),
                                            (70000, 602, 41, 0), (66000, 100, 48, 4)])
@pytest.mark.parametrize("ck", [32, 64])
def test_linear_stream_edges(M, K, C, ld_extra, ck):
    """The streaming forward (linear_stream_kernel, forced; 32- or 64-k
    chunks): W^T in LDS, X
    streamed per 16-row tile with b128 (ld % 4 == 0) or b64 loads (ld = 602,
    the Reddit-train layout); rows past M read zeros, the last chunk's k >= K
    are zeroed (X holds infinities there); M = 70,000 / 66,000 give waves
    more than one tile, so the chunk stream crosses tile boundaries."""
    from sgc_amd import _lib
    from sgc_amd.propagate import linear
    lib = _lib.load()
    g = torch.Generator().manual_seed(M + K + C)
    Xf = torch.full((M, K + ld_extra), float("inf"))
    Xf[:, :K] = torch.randn((M, K), generator=g)
    W = torch.randn((C, K), generator=g) * 0.05
    b = torch.randn(C, generator=g)
    ref = torch.nn.functional.linear(Xf[:, :K].double(), W.double(), b.double())
    tol = 1e-5 * max(1.0, ref.abs().max().item())
    prev_ck = lib.sgc_get_tuning(b"linear_ck")
    _lib.check(lib.sgc_set_tuning(b"linear_kernel", 2), "set_tuning")
    _lib.check(lib.sgc_set_tuning(b"linear_ck", ck), "set_tuning")
    try:
        Xd = Xf.to(DEV)[:, :K]
        Y = linear(Xd, W.to(DEV), b.to(DEV)).cpu().double()
        torch.testing.assert_close(Y, ref, rtol=1e-5, atol=tol)
        Yn = linear(Xd, W.to(DEV), None).cpu().double()
        torch.testing.assert_close(Yn, ref - b.double(), rtol=1e-5, atol=tol)
    finally:
        lib.sgc_set_tuning(b"linear_kernel", 0)
        lib.sgc_set_tuning(b"linear_ck", prev_ck)


@pytest.mark.parametrize("M,K,C,ld_extra", [(129, 602, 41, 6), (300, 33, 17, 1), (257, 31, 3, 1),
                                            (128, 64, 64, 32), (1, 1, 1, 1), (1000, 333, 20, 0),
                                            (70000, 602, 41, 0), (66000, 100, 48, 4),
                                            (4099, 602, 42, 2)])
def test_linear_split_edges(M, K, C, ld_extra):
    """The split-bf16 streaming forward (linear_split_kernel, forced): every
    operand split exactly into three bf16 pieces, six products on
    v_mfma_f32_16x16x32_bf16, within the fp32 tolerance of fp64 torch.  X's
    16-B loads at 8-B (ld = 602, the Reddit-train layout) and 4-B (ld = 333)
    row alignment, 8 lanes per row then a DPP exchange; rows past M read
    zeros; the last chunk's k >= K are zeroed (X holds infinities there);
    class tiles with rows past C; M = 70,000 / 66,000 give waves more than one
    tile, so the chunk stream crosses tile boundaries; C = 42 at K = 602 is
    the largest W image that fits LDS."""
    from sgc_amd import _lib
    from sgc_amd.propagate import linear
    lib = _lib.load()
    g = torch.Generator().manual_seed(M + K + C + 1)
    Xf = torch.full((M, K + ld_extra), float("inf"))
    Xf[:, :K] = torch.randn((M, K), generator=g)
    W = torch.randn((C, K), generator=g) * 0.05
    b = torch.randn(C, generator=g)
    ref = torch.nn.functional.linear(Xf[:, :K].double(), W.double(), b.double())
    tol = 1e-5 * max(1.0, ref.abs().max().item())
    _lib.check(lib.sgc_set_tuning(b"linear_kernel", 5), "set_tuning")
    try:
        Xd = Xf.to(DEV)[:, :K]
        name = lib.sgc_linear_kernel_name(M, K, Xd.stride(0), C, _lib.ptr(Xd)).decode()
        assert name.startswith("linear_split_kernel"), name
        Y = linear(Xd, W.to(DEV), b.to(DEV)).cpu().double()
        torch.testing.assert_close(Y, ref, rtol=1e-5, atol=tol)
        Yn = linear(Xd, W.to(DEV), None).cpu().double()
        torch.testing.assert_close(Yn, ref - b.double(), rtol=1e-5, atol=tol)
    finally:
        lib.sgc_set_tuning(b"linear_kernel", 0)


def test_linear_split_nonfinite_inside_k():
    """VERDICT r05 item 5 / ADVICE: the documented deviation, pinned.  With
    +inf, -inf and NaN features INSIDE the K range (not only in the padding),
    the default GPU forward at M >= 4096 (the split-bf16 kernel) gives NaN in
    exactly those rows' logits -- torch gives +-inf there -- and every other
    row stays within the fp32 tolerance; the fp32 kernel a caller selects with
    sgc_set_tuning("linear_kernel", 2) reproduces torch's non-finite values."""
    from sgc_amd import _lib
    from sgc_amd.propagate import linear
    lib = _lib.load()
    M, K, C = 8192, 602, 41
    g = torch.Generator().manual_seed(5)
    X = torch.randn((M, K), generator=g)
    W = torch.randn((C, K), generator=g) * 0.05
    b = torch.randn(C, generator=g)
    bad = {5: (100, float("inf")), 77: (3, float("-inf")), 1000: (601, float("nan")),
           4097: (0, float("inf"))}
    for r, (k, v) in bad.items():
        X[r, k] = v
    ref = torch.nn.functional.linear(X.double(), W.double(), b.double())
    rows = torch.tensor(sorted(bad))
    good = torch.ones(M, dtype=torch.bool)
    good[rows] = False
    tol = 1e-5 * max(1.0, ref[good].abs().max().item())
    Xd = X.to(DEV)
    name = lib.sgc_linear_kernel_name(M, K, Xd.stride(0), C, _lib.ptr(Xd)).decode()
    assert name.startswith("linear_split_kernel"), name
    Y = linear(Xd, W.to(DEV), b.to(DEV)).cpu().double()
    assert torch.isnan(Y[rows]).all()  # the deviation: NaN, not torch's +-inf
    assert torch.isinf(ref[[5, 77, 4097]]).all()
    torch.testing.assert_close(Y[good], ref[good], rtol=1e-5, atol=tol)
    _lib.check(lib.sgc_set_tuning(b"linear_kernel", 2), "set_tuning")
    try:
        Y32 = linear(Xd, W.to(DEV), b.to(DEV)).cpu().double()
    finally:
        lib.sgc_set_tuning(b"linear_kernel", 0)
    torch.testing.assert_close(Y32[rows], ref[rows], rtol=1e-5, atol=tol, equal_nan=True)
    torch.testing.assert_close(Y32[good], ref[good], rtol=1e-5, atol=tol)


def test_logits_cross_entropy_rejects_out_of_range_labels():
    """a label outside [0, C) that is not ignore_index raises (as
    torch fails on it) instead of returning a NaN loss; ignore_index rows and
    in-range labels pass, and a fixed labels tensor is checked once."""
    from sgc_amd import models
    from sgc_amd.models import SGC
    torch.manual_seed(0)
    model = SGC(32, 5).to(DEV)
    x = torch.randn(64, 32, device=DEV)
    y = torch.randint(0, 5, (64,), device=DEV)
    loss = torch.nn.functional.cross_entropy(model(x), y)
    assert torch.isfinite(loss)
    y_ign = y.clone()
    y_ign[3] = -100
    assert torch.isfinite(torch.nn.functional.cross_entropy(model(x), y_ign))
    for badv in (5, -1, 17):
        y_bad = y.clone()
        y_bad[10] = badv
        with pytest.raises(IndexError, match="out of bounds"):
            torch.nn.functional.cross_entropy(model(x), y_bad)
    n = len(models._checked_labels)
    torch.nn.functional.cross_entropy(model(x), y)
    assert len(models._checked_labels) == n  # cached: no second check


def test_linear_split_precision_vs_fp32_mfma():
    """The split products keep fp32 precision: at the Reddit-train width the
    split kernel's largest error against fp64 is within 2x the fp32 MFMA
    streaming kernel's (both far inside the 1e-5 tolerance), on data with a
    wide exponent range."""
    from sgc_amd import _lib
    from sgc_amd.propagate import linear
    lib = _lib.load()
    g = torch.Generator().manual_seed(5)
    X = torch.randn((8192, 602), generator=g) * torch.exp(2 * torch.randn((8192, 1), generator=g))
    W = torch.randn((41, 602), generator=g) * 0.05
    ref = torch.nn.functional.linear(X.double(), W.double())
    errs = {}
    try:
        for kern in (2, 5):
            _lib.check(lib.sgc_set_tuning(b"linear_kernel", kern), "set_tuning")
            Y = linear(X.to(DEV), W.to(DEV)).cpu().double()
            errs[kern] = ((Y - ref).abs() / (X.double().abs() @ W.double().abs().t())).max().item()
    finally:
        lib.sgc_set_tuning(b"linear_kernel", 0)
    assert errs[5] <= 2 * errs[2] + 1e-8, errs
    assert errs[5] < 1e-6, errs


def test_sgc_model_autograd_matches_torch():
    from sgc_amd.models import SGC, get_model
    torch.manual_seed(0)
    m = SGC(602, 41).to(DEV)
    ref = torch.nn.Linear(602, 41).to(DEV)
    ref.load_state_dict(m.W.state_dict())
    x = torch.randn(500, 602, device=DEV)
    y = torch.randint(0, 41, (500,), device=DEV)
    l1 = torch.nn.functional.cross_entropy(m(x), y)
    l2 = torch.nn.functional.cross_entropy(ref(x), y)
    l1.backward()
    l2.backward()
    torch.testing.assert_close(l1, l2, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(m.W.weight.grad, ref.weight.grad, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(m.W.bias.grad, ref.bias.grad, rtol=1e-4, atol=1e-6)
    assert isinstance(get_model("SGC", 10, 3, cuda=True), SGC)


def _backward_kernel_expected(kernel, K, C):
    if kernel in (0, 3) and C <= 48:
        return "xent_dw_cols"
    if kernel == 2 and K % 2 == 0:
        return "xent_dw_split"
    return "xent_dw_kernel"


@pytest.mark.parametrize("kernel", [0, 1, 2])
@pytest.mark.parametrize("M,K,C", [(1, 3, 2), (140, 1433, 7), (333, 602, 41), (1000, 500, 3),
                                   (4099, 602, 41), (77, 64, 64), (600, 130, 17), (152410, 602, 41),
                                   (5, 601, 1), (225, 34, 48), (100000, 602, 41), (31, 65, 33),
                                   (1537, 129, 16), (20000, 602, 49)])
def test_linear_backward_matches_torch(M, K, C, kernel, request):
    """sgc_linear_backward_f32 (the SGC.forward backward: dW = dY^T X, db =
    sum dY from one read of X) vs fp64 torch, fp32 tolerance; dY a caller's
    [M, C] tensor (classes not a multiple of 16 are masked in the kernel);
    bitwise reproducible run to run.  kernel 0 (auto) takes the split-bf16
    column blocks up to 48 classes (xent_dw_cols_kernel: fewer 32-row steps
    than row ranges, a ragged last step, K not a multiple of 64 or of 4, one
    to three class tiles) and the fp32 slabs above; 1 forces the fp32 slabs;
    2 the split-bf16 slabs (xent_dw_split_kernel; odd K falls back to the
    fp32 slabs)."""
    from sgc_amd import _lib
    from sgc_amd.propagate import linear_backward
    lib = _lib.load()
    _lib.check(lib.sgc_set_tuning(b"backward_kernel", kernel), "set_tuning")
    request.addfinalizer(lambda: lib.sgc_set_tuning(b"backward_kernel", 0))
    name = lib.sgc_linear_backward_kernel_name(M, K, K, C, None).decode()
    assert name.startswith(_backward_kernel_expected(kernel, K, C)), name
    g = torch.Generator().manual_seed(M + 3 * K + C)
    X = torch.randn((M, K), generator=g)
    dY = torch.randn((M, C), generator=g) / M
    dW, db = linear_backward(X.to(DEV), dY.to(DEV))
    wref = dY.double().t() @ X.double()
    bref = dY.double().sum(0)
    torch.testing.assert_close(dW.cpu().double(), wref, rtol=1e-4,
                               atol=1e-5 * max(1e-3, wref.abs().max().item()))
    torch.testing.assert_close(db.cpu().double(), bref, rtol=1e-4,
                               atol=1e-5 * max(1e-3, bref.abs().max().item()))
    dW2, db2 = linear_backward(X.to(DEV), dY.to(DEV))
    assert torch.equal(dW, dW2) and torch.equal(db, db2)
    dW3, none = linear_backward(X.to(DEV), dY.to(DEV), want_bias=False)
    assert none is None and torch.equal(dW, dW3)


@pytest.mark.parametrize("M", [33, 1000, 152410])
def test_linear_backward_cols_edges(M):
    """The column-block backward's edges, each isolated so one element
    would show: (1) dY zero but for the LAST row, K = 602 (the 16-B lane of
    columns 600..603 straddles the end of X: columns 600, 601 must still
    read), so dW must be that row's outer product; (2) X a column slice of a
    wider tensor whose padding columns hold NaN and dY a class slice whose
    padding holds NaN -- the padding is read into columns never stored, or not
    read at all, and no NaN may reach dW or db."""
    from sgc_amd.propagate import linear_backward
    g = torch.Generator().manual_seed(M)
    K, C = 602, 41
    X = torch.randn((M, K), generator=g)
    dY = torch.zeros((M, C))
    dY[-1] = torch.randn(C, generator=g)
    name = _lib_load().sgc_linear_backward_kernel_name(M, K, K, C, None).decode()
    assert name.startswith("xent_dw_cols"), name
    dW, db = linear_backward(X.to(DEV), dY.to(DEV))
    want = dY[-1].double()[:, None] * X[-1].double()[None, :]
    torch.testing.assert_close(dW.cpu().double(), want, rtol=1e-6, atol=0)
    assert torch.equal(db.cpu(), dY[-1])
    Xw = torch.full((M, 640), float("nan"))
    Xw[:, :K] = torch.randn((M, K), generator=g)
    dYw = torch.full((M, 48), float("nan"))
    dYw[:, :C] = torch.randn((M, C), generator=g) / M
    dW, db = linear_backward(Xw.to(DEV)[:, :K], dYw.to(DEV)[:, :C])
    assert torch.isfinite(dW).all() and torch.isfinite(db).all()
    wref = dYw[:, :C].double().t() @ Xw[:, :K].double()
    torch.testing.assert_close(dW.cpu().double(), wref, rtol=1e-4,
                               atol=1e-5 * wref.abs().max().item())
    torch.testing.assert_close(db.cpu().double(), dYw[:, :C].double().sum(0), rtol=1e-4,
                               atol=1e-6)


def _lib_load():
    from sgc_amd import _lib
    return _lib.load()


@pytest.mark.parametrize("M,K,C", [(1, 3, 2), (140, 1433, 7), (333, 602, 41), (1000, 500, 3),
                                   (4099, 602, 41), (77, 64, 64), (600, 130, 17)])
def test_fused_xent_matches_torch(M, K, C):
    """loss, dW, db of the fused training step vs fp64 torch (fp32 tolerance)."""
    from sgc_amd.propagate import linear_xent
    g = torch.Generator().manual_seed(M + K + C)
    X = torch.randn((M, K), generator=g)
    W = torch.randn((C, K), generator=g) * 0.05
    b = torch.randn(C, generator=g) * 0.1
    y = torch.randint(0, C, (M,), generator=g)
    Wd, bd = W.double().requires_grad_(), b.double().requires_grad_()
    ref = torch.nn.functional.cross_entropy(torch.nn.functional.linear(X.double(), Wd, bd), y)
    ref.backward()
    loss, dW, db, logits = linear_xent(X.to(DEV), W.to(DEV), b.to(DEV), y.to(DEV), want_logits=True)
    torch.testing.assert_close(loss.cpu().double(), ref.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dW.cpu().double(), Wd.grad, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(db.cpu().double(), bd.grad, rtol=1e-4, atol=1e-6)
    zref = torch.nn.functional.linear(X.double(), W.double(), b.double())
    torch.testing.assert_close(logits.cpu().double(), zref, rtol=1e-5,
                               atol=1e-5 * max(1.0, zref.abs().max().item()))
    # bitwise reproducible run to run (fixed-order reductions)
    loss2, dW2, db2 = linear_xent(X.to(DEV), W.to(DEV), b.to(DEV), y.to(DEV))
    assert torch.equal(loss, loss2) and torch.equal(dW, dW2) and torch.equal(db, db2)


@pytest.mark.parametrize("M,C,ldl", [(1, 1, 1), (7, 2, 5), (1000, 41, 41), (4099, 64, 64),
                                     (152410, 41, 41), (333, 17, 20), (5000, 3, 3)])
def test_logits_cross_entropy_matches_torch(M, C, ldl):
    """F.cross_entropy on SGCLogits (the reference closures' call, unchanged)
    runs sgc_cross_entropy_f32 / _backward_f32: loss and dlogits vs fp64
    torch (fp32 tolerance), ignore_index rows (-100 and a custom one) left
    out of the mean, strided logits, the incoming gradient scaled on the
    device, bitwise reproducible; a non-plain call (reduction="sum", label
    smoothing) is torch's own."""
    from sgc_amd.models import SGCLogits
    F_ = torch.nn.functional
    g = torch.Generator().manual_seed(M + C)
    base = torch.randn((M, ldl), generator=g) * 3
    y0 = torch.randint(0, C, (M,), generator=g)
    for ign in (-100, 1 % C):
        y = y0.clone()
        if M > 3:
            y[::7] = ign
        ref_x = base[:, :C].double().requires_grad_()
        ref = F_.cross_entropy(ref_x, y, ignore_index=ign)
        (ref * 3).backward()
        full = base.to(DEV).requires_grad_()
        xg = full[:, :C]  # row stride ldl
        logits = xg.as_subclass(SGCLogits)
        loss = F_.cross_entropy(logits, y.to(DEV), ignore_index=ign)
        assert type(loss) is torch.Tensor and loss.grad_fn is not None
        assert "LogitsCrossEntropy" in type(loss.grad_fn).__name__
        (loss * 3).backward()
        # (every row ignored, M = 1: NaN on both sides, as a mean over no rows)
        torch.testing.assert_close(loss.detach().cpu().double(), ref.detach(), rtol=1e-5, atol=1e-6,
                                   equal_nan=True)
        torch.testing.assert_close(full.grad[:, :C].cpu().double(), ref_x.grad, rtol=1e-4,
                                   atol=1e-7, equal_nan=True)
        loss2 = F_.cross_entropy(logits, y.to(DEV), ignore_index=ign)
        assert torch.equal(loss.detach(), loss2.detach()) or torch.isnan(loss2).item()
    s = F_.cross_entropy(base.to(DEV)[:, :C].as_subclass(SGCLogits), y0.to(DEV), reduction="sum")
    assert type(s) is torch.Tensor
    torch.testing.assert_close(s.cpu().double(), F_.cross_entropy(base[:, :C].double(), y0,
                                                                  reduction="sum"),
                               rtol=1e-5, atol=1e-4)


def test_logits_cross_entropy_bad_label_gives_nan():
    """At the C ABI (sgc_cross_entropy_f32, no host check) a label outside
    [0, C) that is not ignore_index makes the loss NaN, without a fault; the
    Python boundary raises before launching (test_logits_cross_entropy_
    rejects_out_of_range_labels)."""
    from sgc_amd import _lib
    from sgc_amd.models import SGCLogits
    lib = _lib.load()
    x = torch.randn(50, 5, device=DEV)
    y = torch.randint(0, 5, (50,), device=DEV)
    y[3] = 9
    loss = torch.empty((), device=DEV)
    inv = torch.empty(1, device=DEV)
    lse = torch.empty(50, device=DEV)
    wsb = lib.sgc_cross_entropy_workspace(50, 5)
    ws = torch.empty(max(1, wsb), dtype=torch.uint8, device=DEV)
    _lib.check(lib.sgc_cross_entropy_f32(_lib.ptr(x), 5, _lib.ptr(y), 50, 5, -100, _lib.ptr(loss),
                                         _lib.ptr(inv), _lib.ptr(lse), _lib.ptr(ws), wsb,
                                         _lib.stream_handle()), "cross_entropy_f32")
    assert torch.isnan(loss).item()
    with pytest.raises(IndexError):
        torch.nn.functional.cross_entropy(x.as_subclass(SGCLogits), y)


def test_unchanged_closure_uses_the_hip_loss():
    """The reference closure as written (citation.py:46-49, reddit.py:55-58:
    zero_grad; F.cross_entropy(model(x), y).backward()) on the drop-in SGC:
    the loss is the HIP kernel's, W / b gradients match nn.Linear + torch's
    loss (fp32 tolerance); eval ops on the logits return plain tensors."""
    from sgc_amd.models import SGC, SGCLogits
    torch.manual_seed(1)
    m = SGC(602, 41).to(DEV)
    ref = torch.nn.Linear(602, 41).to(DEV)
    ref.load_state_dict(m.W.state_dict())
    x = torch.randn(3000, 602, device=DEV)
    y = torch.randint(0, 41, (3000,), device=DEV)
    m.zero_grad()
    out = m(x)
    assert isinstance(out, SGCLogits)
    loss = torch.nn.functional.cross_entropy(out, y)
    assert "LogitsCrossEntropy" in type(loss.grad_fn).__name__
    loss.backward()
    lref = torch.nn.functional.cross_entropy(ref(x), y)
    lref.backward()
    torch.testing.assert_close(loss, lref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(m.W.weight.grad, ref.weight.grad, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(m.W.bias.grad, ref.bias.grad, rtol=1e-4, atol=1e-6)
    preds = out.max(1)[1]
    assert type(preds) is torch.Tensor and type(out.detach().cpu()) is torch.Tensor
    with torch.no_grad():
        lv = torch.nn.functional.cross_entropy(m(x), y)
    torch.testing.assert_close(lv, lref.detach(), rtol=1e-5, atol=1e-5)


def test_fused_loss_trains_like_torch():
    """LBFGS (reddit.py's optimiser) with the fused loss tracks the unfused path."""
    from sgc_amd.models import SGC, sgc_cross_entropy
    torch.manual_seed(0)
    X = torch.randn(3000, 602, device=DEV)
    y = torch.randint(0, 41, (3000,), device=DEV)
    m1 = SGC(602, 41).to(DEV)
    m2 = SGC(602, 41).to(DEV)
    m2.load_state_dict(m1.state_dict())
    losses = []
    for m, fused in ((m1, True), (m2, False)):
        opt = torch.optim.LBFGS(m.parameters(), lr=1)

        def closure():
            opt.zero_grad()
            loss = sgc_cross_entropy(m, X, y) if fused else \
                torch.nn.functional.cross_entropy(m(X), y)
            loss.backward()
            return loss
        for _ in range(2):
            opt.step(closure)
        losses.append(torch.nn.functional.cross_entropy(m(X), y).item())
    assert abs(losses[0] - losses[1]) <= 1e-3 * max(1.0, abs(losses[1])), losses


@pytest.mark.parametrize("name,K,hub", [("norm_n48_F602", 2, None), ("hub1000_F130", 2, 5),
                                        ("norm_n48_F65", 1, None)])
def test_graphed_propagation_bit_exact(tiny_cases, name, K, hub):
    """The K-hop loop captured into a HIP graph (incl. the hub kernel's
    side-stream fork/join when hub=5) replays the reference's bits, for two
    different feature sets through one capture."""
    from sgc_amd.propagate import DeviceCSR, GraphedPropagation
    c = tiny_cases[name]
    csr = DeviceCSR.from_torch(coo_cuda(c))
    X = torch.from_numpy(c["X"]).to(DEV)
    g = GraphedPropagation(csr, X.shape, K, threshold=3 if hub else None, hub_threshold=hub)
    out = g.run(X)
    torch.cuda.synchronize()
    assert bits_equal(out.cpu().numpy(), c[f"Y{K}"])
    X2 = torch.flip(X, dims=[0]).contiguous()
    from sgc_amd.propagate import propagate
    want2 = propagate(csr, X2, K).cpu().numpy()
    out2 = g.run(X2)
    torch.cuda.synchronize()
    assert bits_equal(out2.cpu().numpy(), want2)
    with pytest.raises(RuntimeError):
        g.run(X[:, :1].contiguous())


@pytest.mark.parametrize("name,K", [("norm_n48_F602", 3), ("hub1000_F130", 2), ("norm_n48_F65", 1)])
def test_prepared_loop_replay_bit_exact(tiny_cases, name, K):
    """propagate()'s recorded launch list (sgc_launch_list_*, second call with
    the same shapes / K): the reference's bits, new contents of X picked up,
    OTHER X_0 / X_K tensors of the same layout replayed through the same list
    (X_0 and X_K enter by slot), an X_0 view at another 128-B alignment
    recording its own list, a hop_hook call (the unrecorded loop) agreeing,
    and drop_groups() dropping the lists."""
    from sgc_amd.propagate import DeviceCSR, propagate
    c = tiny_cases[name]
    csr = DeviceCSR.from_torch(coo_cuda(c))
    X = torch.from_numpy(c["X"]).to(DEV)
    out = torch.full_like(X, float("nan"))
    lists = lambda: [k for k in csr._plans if isinstance(k, tuple) and k[0] == "list"]  # noqa: E731
    for _ in range(2):
        propagate(csr, X, K, out=out)
        torch.cuda.synchronize()
        assert bits_equal(out.cpu().numpy(), c[f"Y{K}"])
    assert len(lists()) == 1
    X.copy_(torch.flip(X, dims=[0]))
    want = propagate(csr, X, K, hop_hook=lambda *a: None).cpu().numpy()
    propagate(csr, X, K, out=out)
    torch.cuda.synchronize()
    assert bits_equal(out.cpu().numpy(), want)
    # another X_0 and X_K of the same layout: the same list, their own pointers
    X2 = torch.flip(X, dims=[0]).contiguous()
    out2 = torch.full_like(X, float("nan"))
    propagate(csr, X2, K, out=out2)
    torch.cuda.synchronize()
    assert len(lists()) == 1
    assert bits_equal(out2.cpu().numpy(), c[f"Y{K}"])
    assert bits_equal(out.cpu().numpy(), want)  # the first X_K untouched
    # X_0 one row into a larger buffer: another 128-B alignment class
    n, F = X.shape
    big = torch.zeros((n + 1) * F + 1, device=DEV)
    Xs = big[1:1 + n * F].view(n, F)
    Xs.copy_(torch.from_numpy(c["X"]).to(DEV))
    got = propagate(csr, Xs, K)
    got = propagate(csr, Xs, K)  # replayed
    torch.cuda.synchronize()
    assert bits_equal(got.cpu().numpy(), c[f"Y{K}"])
    assert len(lists()) == 2
    csr.drop_groups()
    assert not lists()


def test_launch_list_per_stream_and_release(tiny_cases):
    """A launch list belongs to its stream: propagate() on a second stream
    records its own (the intermediates are per stream), both replay the
    reference's bits, and DeviceCSR.release_prepared() destroys them (the
    next call records again)."""
    from sgc_amd.propagate import DeviceCSR, propagate
    c = tiny_cases["norm_n48_F602"]
    csr = DeviceCSR.from_torch(coo_cuda(c))
    X = torch.from_numpy(c["X"]).to(DEV)
    lists = lambda: [k for k in csr._plans if isinstance(k, tuple) and k[0] == "list"]  # noqa: E731
    side = torch.cuda.Stream()
    outs = []
    for _ in range(2):
        outs.append(propagate(csr, X, 2))
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            outs.append(propagate(csr, X, 2))
        torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    assert len(lists()) == 2
    for o in outs:
        assert bits_equal(o.cpu().numpy(), c["Y2"])
    csr.release_prepared()
    assert not lists()
    again = propagate(csr, X, 2)
    again = propagate(csr, X, 2)
    torch.cuda.synchronize()
    assert bits_equal(again.cpu().numpy(), c["Y2"]) and len(lists()) == 1


def test_launch_list_abi_errors(tiny_cases):
    """sgc_launch_list_*: unknown handles, bad slots and a slot run without its
    pointer are errors (no launch); destroy frees the handle once; a list of
    one hop with both slots replays bit-exactly."""
    import ctypes
    from sgc_amd import _lib
    from sgc_amd.propagate import DeviceCSR, propagate
    lib = _lib.load()
    c = tiny_cases["norm_n48_F602"]
    csr = DeviceCSR.from_torch(coo_cuda(c))
    X = torch.from_numpy(c["X"]).to(DEV)
    n, F = X.shape
    out = torch.full_like(X, float("nan"))
    s = _lib.stream_handle()
    assert lib.sgc_launch_list_run(987654321, _lib.ptr(X), _lib.ptr(out), s) != 0
    assert lib.sgc_launch_list_destroy(987654321) != 0
    h = ctypes.c_int64(0)
    _lib.check(lib.sgc_launch_list_create(ctypes.byref(h)), "create")
    args = (_lib.ptr(csr.row_ptr), _lib.ptr(csr.col_idx), _lib.ptr(csr.val), 0, n, None, F, None,
            F, F, None, 0, 0, 0, 0)
    assert lib.sgc_launch_list_add_spmm(h.value, *args, 3, 2) != 0      # bad slot
    assert lib.sgc_launch_list_add_spmm(h.value, *args[:-1], 1 << 20, 1, 2) != 0  # unknown flag
    _lib.check(lib.sgc_launch_list_add_spmm(h.value, *args, 1, 2), "add")
    assert lib.sgc_launch_list_run(h.value, None, _lib.ptr(out), s) != 0  # X_0 slot, no X_0
    _lib.check(lib.sgc_launch_list_run(h.value, _lib.ptr(X), _lib.ptr(out), s), "run")
    torch.cuda.synchronize()
    assert bits_equal(out.cpu().numpy(), propagate(csr, X, 1, prepare=False).cpu().numpy())
    _lib.check(lib.sgc_launch_list_destroy(h.value), "destroy")
    assert lib.sgc_launch_list_destroy(h.value) != 0


@pytest.mark.parametrize("r0,r1,th", [(0, 4000, 7), (123, 3001, 0), (0, 4000, 2**31 - 1), (50, 50, 5)])
def test_plan_light_order(r0, r1, th):
    """sgc_plan_light_order: the light rows (degree <= threshold) of the range,
    longest first, ties in row order -- as a stable sort on the host."""
    import ctypes
    from sgc_amd import _lib
    rng = np.random.default_rng(r0 + r1 + th)
    deg = rng.integers(0, 20, 4000)
    rp = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    rp_d = torch.from_numpy(rp).to(DEV)
    out = torch.full((max(1, r1 - r0),), -1, dtype=torch.int32, device=DEV)
    n = ctypes.c_int64(-1)
    lib = _lib.load()
    _lib.check(lib.sgc_plan_light_order(_lib.ptr(rp_d), r0, r1, th, _lib.ptr(out), ctypes.byref(n),
                                        _lib.stream_handle(DEV)), "plan_light_order")
    d = deg[r0:r1]
    light = np.flatnonzero(d <= th)
    want = (light[np.argsort(-d[light], kind="stable")] + r0).astype(np.int32)
    assert n.value == len(want)
    assert np.array_equal(out[:n.value].cpu().numpy(), want)


@pytest.mark.parametrize("r0,r1,th,hub", [(0, 4000, 7, 15), (123, 3001, 0, 0), (0, 4000, 30, 30),
                                          (50, 50, 5, 9), (7, 4000, 2**31 - 2, 2**31 - 2)])
def test_plan_sorted_matches_host_plan(r0, r1, th, hub):
    """sgc_plan_sorted (one device radix sort) lists every row of the range by
    degree, longest first, ties in row order -- the heavy rows of
    sgc_plan_build followed by the light order of sgc_plan_light_order -- and
    counts the heavy rows, the hub rows and the longest row."""
    import ctypes
    from sgc_amd import _lib
    rng = np.random.default_rng(r0 + r1 + th)
    deg = rng.integers(0, 40, 4000)
    rp = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    rp_d = torch.from_numpy(rp).to(DEV)
    n = r1 - r0
    lib = _lib.load()
    out = torch.full((max(1, n),), -1, dtype=torch.int32, device=DEV)
    wb = lib.sgc_plan_sorted_workspace(n)
    ws = torch.empty(max(1, wb), dtype=torch.uint8, device=DEV)
    counts = (ctypes.c_int64 * 3)()
    _lib.check(lib.sgc_plan_sorted(_lib.ptr(rp_d), r0, r1, th, hub, _lib.ptr(out), _lib.ptr(ws), wb,
                                   ctypes.cast(counts, ctypes.c_void_p), _lib.stream_handle(DEV)),
               "plan_sorted")
    d = deg[r0:r1]
    want = (np.argsort(-d, kind="stable") + r0).astype(np.int32)
    assert list(counts) == [int((d > th).sum()), int((d > hub).sum()), int(d.max()) if n else 0]
    assert np.array_equal(out[:n].cpu().numpy(), want)


@pytest.mark.parametrize("n,top", [(20000, 50000), (9000, 5_000_000), (3000, 2047), (2049, 2048),
                                   (70000, 0)])
def test_plan_sorted_multipass(n, top):
    """The plan's radix sort (sort.hip) over several tiles and 1-3 digit
    passes: power-law degrees up to `top` (2,047 and 2,048 sit either side
    of one 11-bit digit; top 0 = every row empty), longest first, ties in row
    order, as a stable host sort."""
    import ctypes
    from sgc_amd import _lib
    rng = np.random.default_rng(n + top)
    deg = np.minimum(rng.pareto(1.2, n) * 3, top).astype(np.int64)
    if top:
        deg[rng.integers(0, n, 3)] = top  # ties at the top
    rp = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    assert rp[-1] < 2**31
    rp_d = torch.from_numpy(rp.astype(np.int32)).to(DEV)
    lib = _lib.load()
    out = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    wb = lib.sgc_plan_sorted_workspace(n)
    ws = torch.empty(max(1, wb), dtype=torch.uint8, device=DEV)
    counts = (ctypes.c_int64 * 3)()
    _lib.check(lib.sgc_plan_sorted(_lib.ptr(rp_d), 0, n, 64, 1024, _lib.ptr(out), _lib.ptr(ws), wb,
                                   ctypes.cast(counts, ctypes.c_void_p), _lib.stream_handle(DEV)),
               "plan_sorted")
    want = np.argsort(-deg, kind="stable").astype(np.int32)
    assert list(counts) == [int((deg > 64).sum()), int((deg > 1024).sum()), int(deg.max())]
    assert np.array_equal(out.cpu().numpy(), want)


@pytest.mark.parametrize("n", [3000, 300000])
def test_ingest_unsorted_multipass(n, oracle):
    """Row-unsorted COO with duplicates over n rows (one or two 11-bit digit
    passes of the ingest's radix sort, many tiles): the CSR is the oracle's
    stable counting sort, bit for bit, and so is one hop."""
    from sgc_amd.propagate import STATUS_ROWS_SORTED, DeviceCSR, spmm
    rng = np.random.default_rng(n)
    nnz = 8 * n
    rows = rng.integers(0, n, nnz)
    cols = rng.integers(0, n, nnz)
    rows[: nnz // 8] = rows[0]  # a hub row with duplicates
    vals = rng.standard_normal(nnz).astype(np.float32)
    idx = torch.from_numpy(np.stack([rows, cols]).astype(np.int64))
    adj = torch.sparse_coo_tensor(idx, torch.from_numpy(vals), (n, n)).to(DEV)
    csr = DeviceCSR.from_torch(adj)
    assert not csr.status & STATUS_ROWS_SORTED
    rp, ci, va = oracle.coo_to_csr(n, n, rows, cols, vals)
    assert np.array_equal(csr.row_ptr.cpu().numpy(), rp)
    assert np.array_equal(csr.col_idx.cpu().numpy(), ci)
    assert bits_equal(csr.val.cpu().numpy(), va)
    X = rng.standard_normal((n, 5)).astype(np.float32)
    y = spmm(csr, torch.from_numpy(X).to(DEV))
    assert bits_equal(y.cpu().numpy(), oracle.spmm_csr(rp, ci, va, X, 0, n))


# ---------------------------------------------------------------------------
# Column groups: one hop as G launches over column ranges (accumulating).

def _split_host(rp, ci, va, n_cols, G):
    """Reference split for sgc_csr_colsplit: group-major arrays, absolute row_ptrs."""
    n = rp.shape[0] - 1
    cuts = [(g * n_cols) // G for g in range(G + 1)]
    rps, cols, vals, base = [], [], [], 0
    row = np.repeat(np.arange(n), np.diff(rp))
    for g in range(G):
        keep = (ci >= cuts[g]) & (ci < cuts[g + 1])
        cnt = np.bincount(row[keep], minlength=n)
        rps.append(base + np.concatenate([[0], np.cumsum(cnt)]))
        cols.append(ci[keep])
        vals.append(va[keep])
        base += int(keep.sum())
    return np.stack(rps).astype(np.int32), np.concatenate(cols), np.concatenate(vals)


@pytest.mark.parametrize("G", [2, 3, 5, 8])
def test_colsplit_matches_host_split(G):
    """sgc_csr_colsplit: each group's row_ptr (absolute offsets) and the
    group-major col / val arrays equal a host split at cuts g * n_cols / G
    (rows with empty groups, a 3,000-nonzero hub, empty rows)."""
    from sgc_amd import graphs
    from sgc_amd.propagate import DeviceCSR
    S = graphs.synthetic_graph("cora", seed=G, n=3000, edges=20000)
    rp = S.row_ptr.astype(np.int64).copy()
    ci, va = S.col_idx.copy(), S.val.copy()
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device=DEV)
    assert csr.cols_ascending
    subs = csr.column_groups(G)
    torch.cuda.synchronize()
    want_rp, want_ci, want_va = _split_host(rp, ci, va, S.n, G)
    for g in range(G):
        assert np.array_equal(subs[g].row_ptr.cpu().numpy(), want_rp[g]), g
    assert np.array_equal(subs[0].col_idx.cpu().numpy(), want_ci)
    assert bits_equal(subs[0].val.cpu().numpy(), want_va)


@pytest.mark.parametrize("G", [2, 3, 4, 8])
def test_column_groups_tiny_cases_bit_exact(tiny_cases, G, monkeypatch):
    """propagate() and sgc_precompute() with G column groups forced: every
    golden case bit-exact; cases whose rows are not strictly ascending (raw
    COO with duplicates / unsorted) run one launch per hop instead."""
    import importlib
    prop_mod = importlib.import_module("sgc_amd.propagate")
    from sgc_amd.propagate import DeviceCSR, column_groups_for, propagate
    monkeypatch.setattr(prop_mod, "COLUMN_GROUPS", G)
    for name, c in tiny_cases.items():
        csr = DeviceCSR.from_torch(coo_cuda(c))
        X = torch.from_numpy(c["X"]).to(DEV)
        if csr.cols_ascending and csr.nnz:
            assert column_groups_for(csr, X.shape[1]) == min(G, csr.n_cols)
        else:
            assert column_groups_for(csr, X.shape[1]) == 1
        for key in sorted(k for k in c if k.startswith("Y") and k != "Y0"):
            out = propagate(csr, X, int(key[1:]))
            torch.cuda.synchronize()
            assert bits_equal(out.cpu().numpy(), c[key]), (name, key, G)


@pytest.mark.parametrize("F", [602, 304, 128, 256])
def test_column_groups_medium_graph_bit_exact(oracle, F):
    """The default rule on a 4.2 M-nonzero graph (two groups at 128 and
    > 256 floats, one at 129-256), forced 1, 3 and 4 groups, split hops (spmm over a row range) and
    the one-launch schedule, the Python hop loop and the native one
    (sgc_propagate_groups_f32): the oracle's bits."""
    from sgc_amd import graphs
    import importlib
    prop_mod = importlib.import_module("sgc_amd.propagate")
    from sgc_amd.propagate import DeviceCSR, column_groups_for, propagate, spmm
    n = 60000
    S = graphs.synthetic_graph("pubmed", seed=11, n=n, edges=2_100_000)
    assert S.nnz >= prop_mod.GROUPS_MIN_NNZ
    X = np.random.default_rng(F).standard_normal((n, F)).astype(np.float32)
    want1 = oracle.spmm_csr(S.row_ptr, S.col_idx, S.val, X, 0, n)
    want2 = oracle.spmm_csr(S.row_ptr, S.col_idx, S.val, want1, 0, n)
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device=DEV)
    Xd = torch.from_numpy(X).to(DEV)
    assert column_groups_for(csr, F) == (1 if 128 < F <= 256 else 2)
    saved = prop_mod.COLUMN_GROUPS
    try:
        for G in (None, 1, 3, 4):
            prop_mod.COLUMN_GROUPS = G
            out = propagate(csr, Xd, 2)
            native = propagate(csr, Xd, 2, native_loop=True)  # sgc_propagate_groups_f32
            part = spmm(csr, Xd, 1000, 37000)
            torch.cuda.synchronize()
            assert bits_equal(out.cpu().numpy(), want2), (F, G)
            assert bits_equal(native.cpu().numpy(), want2), (F, G, "native")
            assert bits_equal(part.cpu().numpy(), want1[1000:37000]), (F, G)
    finally:
        prop_mod.COLUMN_GROUPS = saved
