"""K-hop propagation across GPUs (one process per GPU): four partitions, two
output layouts, and the data-parallel classifier that consumes them.

RowPartitionedPropagator (the north star's layout): each
output row of S.X is an independent FMA chain, so the hot path shards by 1-D
row slicing of S.  Rank p owns the contiguous rows [r_p, r_{p+1}), chosen by
equal nonzero count so power-law hubs do not unbalance the ranks, and
computes those rows of X_{k+1} with the HIP kernel.  Between hops every rank
needs all of X_k (at Reddit/RMAT shape nearly every column is referenced by
every row block), so the exchange is an all-gather of the row blocks per hop
-- RCCL over xGMI with the "nccl" backend (gloo in the CPU tests) -- into a
[P*B, F] buffer (B = the largest block; the rank's CSR carries a second
column-index array in that layout).  Pipelines: one full-width group, feature
groups (group g's all-gather overlaps group g+1's compute), or row chunks
(chunk c all-gathered as soon as it is computed); autotune() picks on the node.

CyclicRowPropagator: row tiles dealt round-robin, so all-gather g of X_k
delivers column group g and hop k+1 consumes it as it arrives (column-group
passes chained by SGC_SPMM_ACCUMULATE, bit-identical to one pass).

TiledPropagator: P = R x C, row blocks x feature blocks (each feature block a
row partition over its R ranks).

FeaturePartitionedPropagator: S.X acts on each feature column independently,
so rank p owns a block of feature columns and runs all K hops over the full S
with no exchange between hops (see its docstring for the measured trade-off).

Output: "replicated" (every rank gets all of X_K) or "sharded" (every rank
keeps its rows of X_K, which is what ShardedSGCTrainer -- the data-parallel
SGC classifier -- consumes; no full X_K is ever materialised).
"""
import contextlib
import os
import time
from dataclasses import dataclass
from typing import Callable, Optional

import numpy as np
import torch
import torch.distributed as dist


def nnz_balanced_bounds(row_ptr, world_size):
    """Row boundaries r_0=0 <= ... <= r_P=N splitting nnz evenly (row_ptr host array)."""
    row_ptr = np.asarray(row_ptr, dtype=np.int64)
    n, nnz = row_ptr.shape[0] - 1, int(row_ptr[-1])
    targets = (np.arange(1, world_size, dtype=np.float64) * nnz / world_size)
    inner = np.searchsorted(row_ptr, targets, side="left").clip(0, n)
    return np.concatenate([[0], inner, [n]]).astype(np.int64)


def equal_row_bounds(n, world_size):
    """r_p = min(p * ceil(n/P), n): equal blocks, the last one shorter."""
    B = max(1, -(-n // world_size))
    return np.minimum(np.arange(world_size + 1, dtype=np.int64) * B, n)


def partition_bounds(row_ptr, world_size, balance="nnz"):
    """Row blocks of the row partition: "nnz" (equal nonzeros, the default:
    power-law hubs and skewed degree ranges do not unbalance the ranks) or
    "rows" (equal rows)."""
    if balance == "nnz":
        return nnz_balanced_bounds(row_ptr, world_size)
    if balance == "rows":
        return equal_row_bounds(len(row_ptr) - 1, world_size)
    raise ValueError(f"balance must be 'nnz' or 'rows', not {balance!r}")


class _StreamDone:
    """A finished-copy handle with the interface of an async collective's
    work object: wait() makes the CURRENT stream wait for the work enqueued on
    `stream` so far (like RCCL's Work.wait())."""
    __slots__ = ("ev", "dev")

    def __init__(self, stream):
        self.dev = stream.device
        self.ev = torch.cuda.Event()
        self.ev.record(stream)

    def wait(self):
        torch.cuda.current_stream(self.dev).wait_event(self.ev)


class _EventsDone:
    """wait() = the current stream waits for the given recorded events (the
    hub-row launches of a split hop, on their own stream)."""
    __slots__ = ("evs",)

    def __init__(self, evs):
        self.evs = evs

    def wait(self):
        cur = torch.cuda.current_stream()
        for ev in self.evs:
            cur.wait_event(ev)


def _local_copy(full, loc):
    """The all-gather of a one-rank group: a copy on the current stream --
    which may be a comm stream, so on the GPU it returns a handle whose wait()
    orders the consumer's stream after the copy (None on the CPU)."""
    full.copy_(loc)
    if full.is_cuda:
        return _StreamDone(torch.cuda.current_stream(full.device))
    return None


def gathered_index(bounds, B, j):
    """Row of global node j in the gathered [P*B, F] exchange buffer: block p
    = the rank owning j lands at rows [p*B, p*B + rows_p)."""
    j = np.asarray(j, dtype=np.int64)
    p = np.searchsorted(bounds, j, side="right") - 1
    return j - bounds[p] + p * B


@dataclass
class ShardCSR:
    """One rank's rows of S (row_ptr rebased to 0).  Two column-index arrays:
    global node ids (hop 1 reads the caller's X_0) and rows of the gathered
    exchange buffer (later hops; identical when the blocks have equal rows)."""
    rank: int
    world_size: int
    bounds: np.ndarray      # [P+1] row boundaries
    row_ptr: torch.Tensor   # int32 [rows+1]
    col_idx: torch.Tensor   # int32 [nnz_local], global ids
    val: torch.Tensor       # float32 [nnz_local]
    n: int
    col_gathered: Optional[torch.Tensor] = None  # int32 [nnz_local], gathered-buffer rows

    @property
    def row_begin(self):
        return int(self.bounds[self.rank])

    @property
    def row_end(self):
        return int(self.bounds[self.rank + 1])

    @property
    def rows(self):
        return self.row_end - self.row_begin

    @property
    def nnz(self):
        return int(self.col_idx.numel())

    @property
    def block(self):
        """Rows per block of the gathered buffer: the largest rank's rows."""
        return max(1, int(np.max(np.diff(self.bounds))))

    @property
    def gathered_rows(self):
        return self.world_size * self.block

    def cols_for(self, layout):
        """Column ids of this rank's CSR for an input layout: "input" (global
        node ids: the caller's X_0), "gathered" (the [P*B, F] exchange buffer)
        or "gathered:RC" (the row-chunked exchange buffer, see
        RowPartitionedPropagator(row_chunks=RC))."""
        if layout == "input":
            return self.col_idx
        rc = int(layout.split(":")[1]) if ":" in layout else 1
        if rc == 1:
            return self.col_gathered
        cache = self.__dict__.setdefault("_chunked_cols", {})
        if rc not in cache:
            Bc = -(-self.block // rc)
            b = torch.as_tensor(self.bounds, dtype=torch.int64, device=self.col_idx.device)
            j = self.col_idx.to(torch.int64)
            q = torch.searchsorted(b, j, right=True) - 1
            i = j - b[q]
            pos = (i // Bc) * (self.world_size * Bc) + q * Bc + i % Bc
            cache[rc] = pos.to(torch.int32)
        return cache[rc]

    def rows_for(self, layout):
        """Rows of the buffer a layout names (its CSR's column count)."""
        if layout == "input":
            return self.n
        rc = int(layout.split(":")[1]) if ":" in layout else 1
        return rc * self.world_size * (-(-self.block // rc))

    @property
    def identity_layout(self):
        """Global row j sits at row j of the gathered buffer (equal blocks)."""
        B = self.block
        return all(int(self.bounds[p]) == min(p * B, self.n) for p in range(self.world_size + 1))


def make_shard(row_ptr, col_idx, val, rank, world_size, device, balance="nnz"):
    """Slice the host CSR (numpy) for `rank` and move it to `device`."""
    row_ptr = np.asarray(row_ptr, dtype=np.int64)
    bounds = partition_bounds(row_ptr, world_size, balance)
    B = max(1, int(np.max(np.diff(bounds))))
    r0, r1 = int(bounds[rank]), int(bounds[rank + 1])
    k0, k1 = int(row_ptr[r0]), int(row_ptr[r1])
    cols = np.asarray(col_idx[k0:k1]).astype(np.int64)
    gcols = gathered_index(bounds, B, cols)
    if world_size * B >= 2**31:
        raise ValueError("gathered exchange buffer exceeds int32 row ids")

    def t(a, dt):
        return torch.from_numpy(np.ascontiguousarray(a)).to(device=device, dtype=dt)

    c = t(cols, torch.int32)
    cg = c if np.array_equal(gcols, cols) else t(gcols, torch.int32)
    return ShardCSR(rank, world_size, bounds, t(row_ptr[r0:r1 + 1] - k0, torch.int32), c,
                    t(np.asarray(val[k0:k1]), torch.float32), int(row_ptr.shape[0] - 1), cg)


def make_shard_device(csr, rank, world_size, balance="nnz"):
    """make_shard for a DeviceCSR without a host round trip: the row bounds
    from a searchsorted over the device row_ptr (P+1 ints come back), the
    rank's col_idx / val as views of the adjacency's own arrays (no copy),
    its row_ptr rebased and its gathered column ids computed on the device.
    The same ShardCSR as make_shard(host arrays) -- tests compare them."""
    rp = csr.row_ptr
    n, nnz = int(csr.n_rows), int(csr.nnz)
    if balance == "nnz":
        targets = (torch.arange(1, world_size, dtype=torch.float64) * nnz / world_size)
        # searchsorted(side="left") of float targets over the int row_ptr,
        # as nnz_balanced_bounds: the first row whose start is >= target
        tgt = torch.ceil(targets).to(torch.int64).to(rp.device)
        inner = torch.searchsorted(rp.to(torch.int64), tgt, right=False).clamp(0, n).cpu()
        bounds = np.concatenate([[0], inner.numpy(), [n]]).astype(np.int64)
    else:
        bounds = partition_bounds(np.zeros(n + 1, np.int64), world_size, balance)
    B = max(1, int(np.max(np.diff(bounds))))
    if world_size * B >= 2**31:
        raise ValueError("gathered exchange buffer exceeds int32 row ids")
    r0, r1 = int(bounds[rank]), int(bounds[rank + 1])
    ks = rp[[r0, r1]].cpu()
    k0, k1 = int(ks[0]), int(ks[1])
    cols = csr.col_idx[k0:k1]
    vals = csr.val[k0:k1]
    row_ptr = (rp[r0:r1 + 1] - k0).to(torch.int32)
    if all(int(bounds[p]) == min(p * B, n) for p in range(world_size + 1)):
        cg = cols  # equal blocks: gathered row j is node j
    else:
        b = torch.as_tensor(bounds, dtype=torch.int64, device=cols.device)
        j = cols.to(torch.int64)
        q = torch.searchsorted(b, j, right=True) - 1
        cg = (j - b[q] + q * B).to(torch.int32)
    return ShardCSR(rank, world_size, bounds, row_ptr, cols, vals, n, cg)


def _default_spmm(shard: ShardCSR, X, out, layout="input", part="all", rows=None):
    """This rank's rows of S.X through the product engine (HIP on ROCm
    tensors, the CPU twin on CPU tensors).  layout: "input" = X is the
    caller's [N, F] X_0 (global column ids), "gathered" = X is the [P*B, F]
    exchange buffer.  part: "all", or the split launch of the multi-GPU
    pipeline -- "light" (every row but the hub rows) and "hub" (only them).
    On the GPU each distinct launch is prepared once (SpmmLaunch) and
    replayed with the current stream: the pipeline's per-step host time
    stays far below its GPU time."""
    from . import _lib
    from .propagate import SPMM_HUB_ONLY, SPMM_NO_HUB, DeviceCSR, SpmmLaunch, spmm
    cache = shard.__dict__.setdefault("_csr_by_layout", {})
    csr = cache.get(layout)
    if csr is None:
        csr = DeviceCSR(shard.rows, shard.rows_for(layout), shard.row_ptr,
                        shard.cols_for(layout), shard.val)
        cache[layout] = csr
    flags = {"all": 0, "light": SPMM_NO_HUB, "hub": SPMM_HUB_ONLY}[part]
    r0, r1 = rows if rows is not None else (0, shard.rows)
    if not X.is_cuda:
        return spmm(csr, X, r0, r1, out=out, flags=flags)
    launches = shard.__dict__.setdefault("_launches", {})
    key = (layout, part, r0, r1, X.data_ptr(), tuple(X.shape), X.stride(0), out.data_ptr(),
           tuple(out.shape), out.stride(0))
    fn = launches.get(key)
    if fn is None:
        if len(launches) > 256:
            launches.clear()
        # keyed by the live tensors' pointers and geometry: no reference kept
        fn = launches[key] = SpmmLaunch(csr, X, out, r0, r1, flags, keep_tensors=False)
    fn(_lib.stream_handle(X.device))
    return out


class RowPartitionedPropagator:
    """X_K = S^K X_0 with S row-sharded over the process group.

    X_0 must be the full [N, F] features on every rank (inputs replicated, as
    the reference loads them).  Each hop computes this rank's rows of S.X_k
    with the HIP kernel (global column ids for hop 1, gathered-buffer rows
    after) and all-gathers them into the [P*B, F] exchange buffer the next
    hop reads (B = the largest block; blocks are nnz-balanced).

    Pipeline per hop (ROCm tensors): the features are processed in groups;
    group g runs as two launches -- every row but the hub rows on the
    caller's stream, the hub rows (long LDS-staged FMA chains) on a hub
    stream -- and group g's all-gather is issued from a comm stream once
    both are done, so the next group's light launch never waits for the hub
    chains and the exchange of group g overlaps the compute of group g+1 and
    the next hop's groups < g.  Bit-exact: every row is still one FMA chain
    per element in CSR order.

    `spmm_fn(shard, X, out, layout, part)` computes the rank's rows; the
    default is the product engine (tests inject the CPU oracle)."""

    def __init__(self, shard: ShardCSR, group=None, spmm_fn: Optional[Callable] = None,
                 group_floats: int = 0, host_staging: bool = False,
                 pad_input: Optional[bool] = None, split_hubs: bool = True,
                 row_chunks: int = 1):
        self.shard = shard
        # Re-lay X_0 into 128-B rows before hop 1?  The copy (all N rows, ~0.2 ms
        # at Reddit shape) beats reading 8-B aligned rows only while this rank's
        # hop-1 share is large: unaligned reads cost +10-18% of that hop
        # (profiles/r01_unaligned_input_sweep.log), so None = pad up to P = 4.
        self.pad_input = pad_input
        self.group = group
        self.spmm_fn = spmm_fn or _default_spmm
        # 0 = one group (full-width launches, no compute/exchange overlap);
        # else 8-B aligned groups of this many floats
        self.group_floats = 0 if int(group_floats) <= 0 else max(2, int(group_floats) // 2 * 2)
        # rehearsal only: gather device buffers through host copies (gloo)
        self.host_staging = host_staging
        self.split_hubs = split_hubs
        # > 1: exchanged hops run full width in this many row chunks, each
        # all-gathered as soon as it is done (one feature group)
        self.row_chunks = max(1, int(row_chunks))
        self._bufs = {}
        self._streams = None
        self._hub_streams = []
        self._event_pool = {}

    def _buf(self, key, shape, like):
        b = self._bufs.get(key)
        if b is None or tuple(b.shape) != tuple(shape) or b.device != like.device:
            b = torch.empty(shape, dtype=torch.float32, device=like.device)
            self._bufs[key] = b
        return b

    def _all_gather(self, full, loc):
        if self.shard.world_size == 1:  # the exchange of one rank is a copy
            return _local_copy(full, loc)
        if not self.host_staging:
            return dist.all_gather_into_tensor(full, loc, group=self.group, async_op=True)
        h_full = torch.empty(full.shape, dtype=full.dtype)
        dist.all_gather_into_tensor(h_full, loc.cpu(), group=self.group)
        full.copy_(h_full)
        return None

    def autotune(self, X0, K, output="sharded", candidates=(0, "r4", 256, 128), reps=2):
        """Pick group_floats by timing whole propagations (collective: every
        rank must call it with the same arguments).  The best grouping depends
        on the exchange rate, which only the node knows: narrower groups hide
        more of the all-gather behind compute but each group launch re-reads
        the CSR and pays a launch tail -- on one GPU a rank's P=8 step takes
        1.7 ms as one full-width group (0) and 2.3-2.9 ms in 128-float groups
        (profiles/r02/p8_rehearsal_*.log), so only a slow exchange favours
        groups.  Each candidate's time is the max over ranks, so every rank
        picks the same width (the all-gathers' shapes must agree).
        Returns {group_floats: seconds per propagation}."""
        import time

        def sync():
            if X0.is_cuda:
                torch.cuda.synchronize(X0.device)
            dist.barrier(group=self.group)

        on_dev = X0.is_cuda and dist.get_backend(self.group) == "nccl"
        times = {}
        for gf in candidates:
            # an int = feature-group width (0: one group); "rN" = one group in
            # N row chunks per exchanged hop
            if isinstance(gf, str) and gf.startswith("r"):
                self.group_floats, self.row_chunks = 0, int(gf[1:])
            else:
                self.group_floats = 0 if int(gf) <= 0 else max(2, int(gf) // 2 * 2)
                self.row_chunks = 1
            self._bufs.clear()
            self.propagate(X0, K, output=output)  # warm-up: buffers, plans
            sync()
            t0 = time.perf_counter()
            for _ in range(reps):
                self.propagate(X0, K, output=output)
            sync()
            t = torch.tensor([(time.perf_counter() - t0) / reps], dtype=torch.float64,
                             device=X0.device if on_dev else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
            times[gf] = float(t.item())
        best = min(times, key=lambda g: (times[g], str(g)))
        if isinstance(best, str):
            self.group_floats, self.row_chunks = 0, int(best[1:])
        else:
            self.group_floats = 0 if int(best) <= 0 else max(2, int(best) // 2 * 2)
            self.row_chunks = 1
        self._bufs.clear()
        return times

    def _compute(self, X, out, layout, split, key=None, rows=None):
        """One group's (or row chunk's) local SpMM: (light event, hub event) on
        the GPU when the launch is split, else (None, None) after one launch."""
        kw = {} if rows is None else {"rows": rows}
        n_rows = self.shard.rows if rows is None else rows[1] - rows[0]
        if not split:
            if n_rows:
                self.spmm_fn(self.shard, X, out, layout, "all", **kw)
            return None, None
        main = torch.cuda.current_stream(X.device)
        hub_s = self._hub_stream(key[-1] if isinstance(key[-1], int) else 0, X.device)
        ready, ev_l, ev_h = self._events(key)
        ready.record(main)
        # hub rows first: their CU-sized workgroups must be queued before the
        # light launch fills every CU, or their ~0.3 ms chains start only as
        # the light kernel drains and end past it (+0.3 ms per hop at world 1,
        # profiles/r03 rccl1 logs) -- launch_spmm's own fork orders them so too
        hub_s.wait_event(ready)
        with torch.cuda.stream(hub_s):
            if n_rows:
                self.spmm_fn(self.shard, X, out, layout, "hub", **kw)
        ev_h.record(hub_s)
        if n_rows:
            self.spmm_fn(self.shard, X, out, layout, "light", **kw)
        ev_l.record(main)
        return ev_l, ev_h

    def _issue_gather(self, full, loc, ev_l, ev_h, split):
        if split:
            comm = self._streams[1]
            comm.wait_event(ev_l)
            comm.wait_event(ev_h)
            with torch.cuda.stream(comm):
                return self._all_gather(full, loc)
        return self._all_gather(full, loc)

    def _propagate_row_chunks(self, X0, K, out, output, F, Fp, split):
        """Exchanged hops at full width in RC row chunks: chunk c of every rank
        is all-gathered into rows [c*P*Bc, (c+1)*P*Bc) of the exchange buffer
        as soon as it is computed, so the hop's exchange overlaps its own
        later chunks (the next hop needs all of X_k: every row reads every
        column block, in column order).  Layout "gathered:RC" remaps the
        columns (ShardCSR.cols_for).  X0 is the caller's [N, F] or its
        128-B-row copy [N, Fp]; exchanged buffers are [., Fp] (pad columns
        carry don't-care values and are never returned)."""
        s = self.shard
        n = X0.shape[0]
        RC = self.row_chunks
        Bc = -(-s.block // RC)
        PB = RC * s.world_size * Bc
        src, layout, works = X0, "input", []
        K_ex = K - 1 if output == "sharded" else K
        for h in range(K_ex):
            for w in works:
                if w is not None:
                    w.wait()  # all of X_h has arrived
            W = min(src.shape[1], Fp)
            full = self._buf(("cfull", h & 1), (PB, Fp), X0)
            works = []
            for c in range(RC):
                lo, hi = c * Bc, min((c + 1) * Bc, s.rows)
                loc = self._buf(("cloc", h & 1, c), (Bc, Fp), X0)
                ev_l = ev_h = None
                if hi > lo:
                    ev_l, ev_h = self._compute(src[:, :W], loc[:hi - lo, :W], layout, split,
                                               key=("chunk", h, c), rows=(lo, hi))
                elif split:
                    _, ev_l, ev_h = self._events(("chunk", h, c))
                    main = torch.cuda.current_stream(X0.device)
                    ev_l.record(main)
                    ev_h.record(main)
                seg = full[c * s.world_size * Bc:(c + 1) * s.world_size * Bc]
                works.append(self._issue_gather(seg, loc, ev_l, ev_h, split))
            src, layout = full, f"gathered:{RC}"
        for w in works:
            if w is not None:
                w.wait()
        if output == "sharded":
            if out is None:
                out = torch.empty((s.rows, F), dtype=torch.float32, device=X0.device)
            if s.rows:
                _, ev_h = self._compute(src[:, :F], out, layout, split, key=("chunk", "last"))
                if ev_h is not None:
                    torch.cuda.current_stream(X0.device).wait_event(ev_h)
            return out
        if out is None:
            out = torch.empty((n, F), dtype=torch.float32, device=X0.device)
        for q in range(s.world_size):
            r0, r1 = int(s.bounds[q]), int(s.bounds[q + 1])
            for c in range(RC):
                a, b = r0 + c * Bc, min(r0 + (c + 1) * Bc, r1)
                if b > a:
                    base = c * s.world_size * Bc + q * Bc
                    out[a:b].copy_(src[base:base + (b - a), :F])
        return out

    def _hub_stream(self, gi, device):
        """One stream per feature group for its hub rows: the hub kernels of a
        hop's groups run concurrently (each is bounded by its longest row's
        FMA chain, ~0.3 ms for the 47,857-nonzero row), not one after another."""
        hs = self._hub_streams
        while len(hs) <= gi:
            hs.append(torch.cuda.Stream(device=device))
        return hs[gi]

    def _events(self, key):
        """(input ready, light done, hub done) events of one launch slot, made
        once and re-recorded every step (a wait enqueued earlier keeps the
        state it saw)."""
        ev = self._event_pool.get(key)
        if ev is None:
            ev = self._event_pool[key] = (torch.cuda.Event(), torch.cuda.Event(),
                                          torch.cuda.Event())
        return ev

    def propagate(self, X0, K, out=None, output="replicated"):
        """output="replicated": the full X_K [N, F] on every rank (one more
        all-gather after the last hop).  output="sharded": this rank's rows
        [row_begin, row_end) of X_K as a [rows, F] tensor -- the layout a
        data-parallel classifier consumes (sgc_amd.distributed.
        ShardedSGCTrainer); the last hop then needs no exchange."""
        s = self.shard
        n, F = X0.shape
        if output not in ("replicated", "sharded"):
            raise ValueError(f"output must be 'replicated' or 'sharded', not {output!r}")
        if K <= 0:
            return X0 if output == "replicated" else X0[s.row_begin:s.row_end]
        split = X0.is_cuda and self.split_hubs and not self.host_staging
        if split and self._streams is None:
            self._streams = (torch.cuda.Stream(device=X0.device),
                             torch.cuda.Stream(device=X0.device))
        Fp = F
        if X0.is_cuda:
            from . import _lib
            from .propagate import aligned_ld
            Fp = aligned_ld(F)  # exchanged buffers keep 128-B rows either way
            pad = self.pad_input if self.pad_input is not None else s.world_size <= 4
            if pad:
                Xa = self._buf("x0", (n, Fp), X0)  # 128-B rows (propagate() does the same)
                _lib.check(_lib.load().sgc_pad_rows_f32(
                    _lib.ptr(X0), X0.stride(0), _lib.ptr(Xa), Fp, n, F,
                    _lib.stream_handle(X0.device)), "pad_rows_f32")
                X0 = Xa
        if self.row_chunks > 1 and s.world_size > 1:
            return self._propagate_row_chunks(X0, K, out, output, F, Fp, split)
        # one group on a single rank: nothing to overlap, and each extra group
        # re-reads the CSR and adds a launch tail (+35% at world 1, r01)
        gf = self.group_floats if s.world_size > 1 and self.group_floats > 0 else Fp
        groups = [(a, min(Fp, a + gf)) for a in range(0, Fp, gf)]
        src = [X0[:, a:min(b, X0.shape[1])] for a, b in groups]  # unpadded: last one narrower
        layout = "input"
        works = [None] * len(groups)
        if output == "sharded":
            K_ex = K - 1  # hops whose output is exchanged
            if out is None:
                out = torch.empty((s.rows, F), dtype=torch.float32, device=X0.device)
        else:
            K_ex = K
        PB = s.gathered_rows
        for h in range(K_ex):
            par = h & 1
            new_works, gathered = [], []
            for gi, (a, b) in enumerate(groups):
                if works[gi] is not None:
                    works[gi].wait()  # this hop's input group has arrived (stream wait)
                full = self._buf(("full", par, gi), (PB, b - a), X0)
                # one rank: its block IS the gathered buffer (no exchange copy)
                loc = (full if s.world_size == 1 else
                       self._buf(("local", par, gi), (s.block, b - a), X0))
                ev_l, ev_h = self._compute(src[gi], loc[:s.rows, :src[gi].shape[1]], layout,
                                           split, key=(h, gi))
                if s.world_size == 1:
                    new_works.append(_EventsDone([ev_h]) if ev_h is not None else None)
                else:
                    new_works.append(self._issue_gather(full, loc, ev_l, ev_h, split))
                gathered.append(full)
            works, src, layout = new_works, gathered, "gathered"
        if output == "sharded":
            # last hop: each group straight into this rank's rows of X_K
            hub_events = []
            for gi, (a, b) in enumerate(groups):
                if works[gi] is not None:
                    works[gi].wait()
                bb = min(b, F)
                if bb > a:
                    _, ev_h = self._compute(src[gi][:, :bb - a], out[:, a:bb], layout, split,
                                            key=("last", gi))
                    if ev_h is not None:
                        hub_events.append(ev_h)
            if hub_events:
                main = torch.cuda.current_stream(X0.device)
                for ev in hub_events:
                    main.wait_event(ev)
            return out
        for w in works:
            if w is not None:
                w.wait()
        if out is None:
            out = torch.empty((n, F), dtype=torch.float32, device=X0.device)
        # compact the gathered blocks (row p*B + i -> global row bounds[p] + i)
        for gi, (a, b) in enumerate(groups):
            bb = min(b, F)
            if bb <= a:
                continue
            if s.identity_layout:  # block p already sits at rows [p*B, ...)
                out[:, a:bb].copy_(src[gi][:n, :bb - a])
                continue
            for p in range(s.world_size):
                r0, r1 = int(s.bounds[p]), int(s.bounds[p + 1])
                if r1 > r0:
                    out[r0:r1, a:bb].copy_(src[gi][p * s.block:p * s.block + (r1 - r0), :bb - a])
        return out


# ---------------------------------------------------------------------------
# Cyclic row partition with column-ordered exchange (SURVEY.md 8(e) overlap).

@dataclass
class CyclicShard:
    """One rank's rows of S under the cyclic tiling of CyclicRowPropagator.

    Rows are cut into tiles of `tile` consecutive rows; tile t*P + p goes to
    rank p, for rounds t = 0..T-1, T = G*Tg (rows past n are empty padding).
    Rank p's local row t*tile + i is global row (t*P + p)*tile + i, so its
    local rows are in ascending global order, and the rounds of column group g
    (t in [g*Tg, (g+1)*Tg)) cover the contiguous global range
    [g*Tg*P*tile, (g+1)*Tg*P*tile) -- held by ALL ranks in equal parts.

    csr_input: the rank's rows with global column ids (hop 1 reads X_0).
    sub[g]: the same rows restricted to column group g, with columns remapped
    to rows of the exchange buffer (see gathered_index); each row's nonzeros of
    group g are a contiguous run of its CSR-ordered nonzeros, so passes over
    g = 0, 1, ... in order are the row's FMA chain in CSR order."""
    rank: int
    world_size: int
    n: int
    tile: int
    groups: int
    rounds_per_group: int
    global_rows: np.ndarray          # int64 [T*tile] global id of each local row
    n_valid: int                     # local rows with global id < n (a prefix)
    csr_input: "object"              # DeviceCSR over [T*tile] rows, global columns
    sub: list                        # [G] DeviceCSR over [T*tile] rows, gathered columns
    nnz: int

    @property
    def rows(self):
        """Local rows, padding included (every launch covers all of them)."""
        return int(self.global_rows.shape[0])

    @property
    def group_rows(self):
        """Local rows per column group (= rows each rank sends per all-gather)."""
        return self.rounds_per_group * self.tile

    @property
    def gathered_rows(self):
        return self.world_size * self.rows


def cyclic_layout(n, world_size, tile, groups):
    """(rounds per group Tg, rounds T = groups*Tg) covering n rows."""
    tiles = max(1, -(-n // tile))
    rounds = -(-tiles // world_size)
    Tg = max(1, -(-rounds // groups))
    return Tg, groups * Tg


def cyclic_gathered_index(j, world_size, tile, Tg):
    """Exchange-buffer row of global node j: group g's all-gather lands rank
    q's Tg tiles at rows [(g*P + q)*Tg*tile, ...), tile t' (within the group)
    at offset t'*tile."""
    j = np.asarray(j, dtype=np.int64)
    P, b = world_size, tile
    t = j // (P * b)
    q = (j // b) % P
    i = j % b
    g, tl = t // Tg, t % Tg
    return ((g * P + q) * Tg + tl) * b + i


def make_cyclic_shard(row_ptr, col_idx, val, rank, world_size, device, tile=64, groups=4):
    """Host (numpy) slicing of S for `rank` under the cyclic tiling, moved to
    `device` as DeviceCSRs (hop-1 CSR + one per column group)."""
    from .propagate import DeviceCSR
    row_ptr = np.asarray(row_ptr, dtype=np.int64)
    n = int(row_ptr.shape[0] - 1)
    P, b, G = int(world_size), int(tile), int(groups)
    if P < 1 or b < 1 or G < 1:
        raise ValueError("world_size, tile and groups must be >= 1")
    Tg, T = cyclic_layout(n, P, b, G)
    if P * T * b >= 2**31:
        raise ValueError("cyclic exchange buffer exceeds int32 row ids")
    t = np.arange(T, dtype=np.int64)
    starts = (t * P + rank) * b                         # global first row of each local tile
    grows = (starts[:, None] + np.arange(b, dtype=np.int64)[None, :]).reshape(-1)
    valid = grows < n
    n_valid = int(valid.sum())
    gv = grows[:n_valid]                                # valid local rows are a prefix
    deg = np.zeros(T * b, dtype=np.int64)
    deg[:n_valid] = row_ptr[gv + 1] - row_ptr[gv]
    lrp = np.zeros(T * b + 1, dtype=np.int64)
    np.cumsum(deg, out=lrp[1:])
    nnz = int(lrp[-1])
    # nonzeros of each local tile are one contiguous range of the global CSR
    t0 = np.minimum(starts, n)
    t1 = np.minimum(starts + b, n)
    k0, k1 = row_ptr[t0], row_ptr[t1]
    lens = k1 - k0
    idx = np.repeat(k0 - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens) + \
        np.arange(nnz, dtype=np.int64)
    cols = np.asarray(col_idx)[idx].astype(np.int64)
    vals = np.asarray(val)[idx].astype(np.float32)
    del idx
    gcols = cyclic_gathered_index(cols, P, b, Tg)
    grp = cols // (P * b * Tg)                          # column group of each nonzero
    local_row = np.repeat(np.arange(T * b, dtype=np.int64), deg)
    if G > 1 and nnz > 1:
        # the passes visit groups 0, 1, ...: a row's CSR order must not go back
        # to an earlier group (any column-sorted CSR -- the reference's scipy S
        # -- qualifies; storage-order COO with unsorted rows may not)
        back = (np.diff(grp) < 0) & (local_row[1:] == local_row[:-1])
        if back.any():
            i = int(local_row[1:][back][0])
            raise ValueError(
                f"CyclicRowPropagator: row {int(grows[i])}'s nonzeros are not in ascending "
                f"column-group order, so column-group passes would reorder its FMA chain; "
                f"use groups=1 or another partition for this CSR")
    counts = np.bincount(local_row * G + grp, minlength=T * b * G).reshape(T * b, G)
    del local_row
    order = np.argsort(grp, kind="stable")              # group-major, CSR order within

    def dev(a, dt):
        return torch.from_numpy(np.ascontiguousarray(a)).to(device=device, dtype=dt)

    csr_input = DeviceCSR(T * b, n, dev(lrp, torch.int32), dev(cols, torch.int32),
                          dev(vals, torch.float32))
    sub, off = [], 0
    for g in range(G):
        rp = np.zeros(T * b + 1, dtype=np.int64)
        np.cumsum(counts[:, g], out=rp[1:])
        sel = order[off:off + int(rp[-1])]
        off += int(rp[-1])
        sub.append(DeviceCSR(T * b, P * T * b, dev(rp, torch.int32), dev(gcols[sel], torch.int32),
                             dev(vals[sel], torch.float32)))
    return CyclicShard(rank, P, n, b, G, Tg, grows, n_valid, csr_input, sub, nnz)


def _pad_columns_allocated(t):
    """Columns [F, round4(F)) of every row of the 2-D view t lie inside its
    storage (F % 4 != 0 only: otherwise there is nothing to pad)."""
    rows, F = t.shape
    F4 = -(-F // 4) * 4
    if F4 == F or rows == 0 or t.stride(1) != 1 or t.stride(0) < F4:
        return False
    end = t.storage_offset() + (rows - 1) * t.stride(0) + F4
    return end * t.element_size() <= t.untyped_storage().nbytes()


def _cyclic_spmm(csr, X, out, rows, accumulate, part="all", thresholds=(None, None),
                 own=(False, False)):
    """Rows [r0, r1) of csr . X into out[r0:r1] through the product engine;
    accumulate = continue the chains stored in out (SPMM_ACCUMULATE); part =
    "all", or the split launch "light" (all but the hub rows) / "hub";
    thresholds = (heavy, hub) row-length thresholds of the plan; own = (X, out)
    are the propagator's own 128-B-row buffers, whose pad columns the kernel
    may read / overwrite (never a caller's tensor: a column view of a wider
    caller buffer would get its neighbouring columns clobbered)."""
    from . import _lib
    from .propagate import (SPMM_ACCUMULATE, SPMM_HUB_ONLY, SPMM_NO_HUB, SPMM_X_PADDED,
                            SPMM_Y_PADDED, SpmmLaunch, spmm)
    r0, r1 = rows
    th, hub = thresholds
    flags = (SPMM_ACCUMULATE if accumulate else 0) | \
        {"all": 0, "light": SPMM_NO_HUB, "hub": SPMM_HUB_ONLY}[part]
    if X.shape[1] < out.shape[1]:
        raise ValueError("output wider than input")
    if not X.is_cuda:
        return spmm(csr, X, r0, r1, out=out[r0:r1], flags=flags, threshold=th, hub_threshold=hub)
    # the engine's own buffers have 128-B rows: let the kernel use 16-B lanes
    # (columns [F, round4(F)) of every row allocated; their values unused)
    if own[0] and _pad_columns_allocated(X):
        flags |= SPMM_X_PADDED
    if own[1] and _pad_columns_allocated(out):
        flags |= SPMM_Y_PADDED
    launches = csr.__dict__.setdefault("_launches", {})
    key = (r0, r1, flags, th, hub, X.data_ptr(), tuple(X.shape), X.stride(0), out.data_ptr(),
           tuple(out.shape), out.stride(0))
    fn = launches.get(key)
    if fn is None:
        if len(launches) > 256:
            launches.clear()
        # keyed by the live tensors' pointers and geometry, so the entry holds
        # no reference to them (a caller's X0 / out is never pinned)
        fn = launches[key] = SpmmLaunch(csr, X, out[r0:r1], r0, r1, flags, threshold=th,
                                        hub_threshold=hub, keep_tensors=False)
    fn(_lib.stream_handle(X.device))
    return out


class CyclicRowPropagator:
    """X_K = S^K X_0 with S's rows dealt out in tiles, round-robin over the
    ranks, and the next hop consuming the exchange column group by column
    group as it arrives -- SURVEY.md 8(e)'s overlap, built for a point-to-
    point xGMI mesh.

    Why cyclic.  Hop k+1 may add row i's nonzeros only in CSR (ascending
    column) order, so it can start on the part of X_k whose columns come
    first.  With contiguous row blocks the first columns all live on rank 0,
    and delivering them first would leave 6 of every GPU's 7 links idle.
    With tiles dealt round-robin, the first Tg*P tiles of X_k -- the first
    column group -- are spread evenly over ALL ranks: the exchange is G
    ordinary all-gathers (every link busy), and all-gather g delivers exactly
    column group g.

    Per hop (GPU; G = `groups`):
      * hop 1 reads the caller's X_0 (global column ids) in one pass;
      * hop k >= 2 runs G passes over the rank's rows: pass g uses only the
        nonzeros of column group g, waits only for all-gather g of X_{k-1},
        and continues the FMA chains pass g-1 stored (SGC_SPMM_ACCUMULATE:
        one fp32 store/load per element between passes -- exact, so the
        result is bit-identical to one pass);
      * when the hop's output is exchanged, its final pass runs in G row
        chunks (local rows of column group c) and all-gather c is issued on
        the comm stream as soon as chunk c is done -- so the exchange of X_k
        overlaps hop k's own tail AND hop k+1's passes over earlier groups.
    Costs: the accumulator round trip (2 x 4F bytes per row per extra pass)
    and G launches per hop instead of one; the gain is that the next hop's
    passes read X from one column group at a time (1/G of X_k live: better
    L2 / Infinity Cache reuse than a full-width pass over all of X_k).

    output="sharded": this rank's rows of X_K, in ascending global order,
    global ids in `row_index` (valid rows only).  output="replicated": X_K
    [N, F] on every rank.  spmm_fn(csr, X, out, rows, accumulate, part,
    thresholds, own=(X is ours, out is ours)) computes out[rows] (default: the HIP engine on ROCm tensors, the CPU twin
    on CPU tensors).

    Heavy/hub row thresholds come from the rank's whole CSR (its nonzeros and
    the width), not from each chunk or pass: sized per chunk, the hub
    threshold (nnz / 1024) would fall to ~1k nonzeros at P = 8 and turn
    thousands of mid-size rows into CU-sized hub workgroups (hop 1's hub
    launches then ran 1.1-1.8 ms beside 0.6 ms of light rows).

    Hub rows: hop 1's row chunks run as split launches -- the hub rows of
    every chunk first, on a hub stream, then the light rows chunk by chunk on
    the compute stream; all-gather c waits for both halves of chunk c -- so a
    0.3-ms hub chain does not hold back the next chunk, and the hub
    workgroups (a CU's LDS each) are not starved by light chunks issued
    before them.  The column-group passes keep each launch's hub kernel joined: a row
    that is a hub of pass g may be a light row of pass g+1, which must not
    start on it before pass g's chain has stored."""

    def __init__(self, row_ptr, col_idx, val, rank, world_size, device, group=None,
                 tile=64, groups=4, host_staging=False, spmm_fn: Optional[Callable] = None,
                 pad_input: Optional[bool] = None):
        self.shard = make_cyclic_shard(row_ptr, col_idx, val, rank, world_size, device, tile,
                                       groups)
        self.group = group
        self.host_staging = host_staging
        self.spmm_fn = spmm_fn or _cyclic_spmm
        self.pad_input = pad_input
        self._bufs = {}
        self._comm = None
        self._hub = None
        self._events = {}
        self._th = (None, None)

    @property
    def row_index(self):
        return self.shard.global_rows[:self.shard.n_valid]

    def _buf(self, key, shape, like):
        b = self._bufs.get(key)
        if b is None or tuple(b.shape) != tuple(shape) or b.device != like.device:
            b = torch.empty(shape, dtype=torch.float32, device=like.device)
            self._bufs[key] = b
        return b

    def _all_gather(self, full, loc):
        if self.shard.world_size == 1:
            return _local_copy(full, loc)
        if not self.host_staging:
            return dist.all_gather_into_tensor(full, loc, group=self.group, async_op=True)
        h = torch.empty(full.shape, dtype=full.dtype)
        dist.all_gather_into_tensor(h, loc.cpu(), group=self.group)
        full.copy_(h)
        return None

    def _event(self, key):
        ev = self._events.get(key)
        if ev is None:
            ev = self._events[key] = torch.cuda.Event()
        return ev

    def _issue(self, full, loc, key, hub_done=None):
        """All-gather loc -> full once the work enqueued so far on the current
        stream (and hub_done, if given) is done (GPU: from the comm stream,
        asynchronously)."""
        if not full.is_cuda or self.host_staging:
            return self._all_gather(full, loc)
        ev = self._event(("ready",) + key)
        ev.record(torch.cuda.current_stream(full.device))
        self._comm.wait_event(ev)
        if hub_done is not None:
            self._comm.wait_event(hub_done)
        with torch.cuda.stream(self._comm):
            return self._all_gather(full, loc)

    def _thresholds(self, F):
        """(heavy, hub) thresholds for every launch of this rank at width F."""
        from .propagate import (DEFAULT_HEAVY_THRESHOLD, DEFAULT_HUB_THRESHOLD,
                                auto_heavy_threshold, auto_hub_threshold)
        th = DEFAULT_HEAVY_THRESHOLD
        if th is None:
            th = auto_heavy_threshold(self.shard.nnz, F)
        hub = DEFAULT_HUB_THRESHOLD
        if hub is None:
            hub = auto_hub_threshold(self.shard.nnz, th)
        return int(th), int(max(hub, th))

    def _hub_first(self, csr, X, out, chunks, h, own):
        """Hop 1's hub rows, issued before any of its light chunks: one
        HUB_ONLY launch per row chunk on the hub stream (after the work already
        on the current stream), so their CU-sized workgroups are placed before
        the light chunks fill the machine.  Returns each chunk's done event."""
        main = torch.cuda.current_stream(X.device)
        ready = self._event(("in", h))
        ready.record(main)
        self._hub.wait_event(ready)
        done = []
        with torch.cuda.stream(self._hub):
            for c, rows in enumerate(chunks):
                self.spmm_fn(csr, X, out, rows, False, "hub", self._th, own=own)
                ev = self._event(("hub", h, c))
                ev.record(self._hub)
                done.append(ev)
        return done

    def propagate(self, X0, K, out=None, output="sharded"):
        s = self.shard
        n, F = X0.shape
        if n != s.n:
            raise ValueError(f"X0 has {n} rows, S has {s.n}")
        if output not in ("replicated", "sharded"):
            raise ValueError(f"output must be 'replicated' or 'sharded', not {output!r}")
        if K <= 0:
            return X0 if output == "replicated" else X0[torch.as_tensor(self.row_index,
                                                                       device=X0.device)]
        Fp = F
        src_own = False  # X0 is the caller's tensor (never pad-written / pad-read)
        if X0.is_cuda:
            from . import _lib
            from .propagate import aligned_ld
            Fp = aligned_ld(F)
            if self._comm is None:
                self._comm = torch.cuda.Stream(device=X0.device)
                self._hub = torch.cuda.Stream(device=X0.device)
            pad = self.pad_input if self.pad_input is not None else s.world_size <= 4
            if pad:
                Xa = self._buf("x0", (n, Fp), X0)
                _lib.check(_lib.load().sgc_pad_rows_f32(
                    _lib.ptr(X0), X0.stride(0), _lib.ptr(Xa), Fp, n, F,
                    _lib.stream_handle(X0.device)), "pad_rows_f32")
                X0 = Xa
                src_own = True
        G, R, GR = s.groups, s.rows, s.group_rows
        PGR = s.world_size * GR                   # exchange-buffer rows per group
        self._th = self._thresholds(F)
        src, works = X0, None
        for h in range(K):
            last = h == K - 1
            exchanged = not last or output == "replicated"
            if exchanged:
                dst = self._buf(("loc", h & 1), (R, Fp), X0)
                full = self._buf(("full", h & 1), (G * PGR, Fp), X0)
            else:
                if out is None:
                    out = torch.empty((R, F), dtype=torch.float32, device=X0.device)
                elif tuple(out.shape) != (R, F):
                    raise ValueError(f"out must be [{R}, {F}] (local rows, padding included)")
                dst = out
            W = min(dst.shape[1], src.shape[1])
            own = (src_own, exchanged)  # dst = out (a caller's) on the last, unexchanged hop
            passes = [(s.csr_input, None)] if h == 0 else [(s.sub[g], g) for g in range(G)]
            new_works = []
            for pi, (csr, g) in enumerate(passes):
                if g is not None and works is not None and works[g] is not None:
                    works[g].wait()               # column group g of X_{h} has arrived
                acc = pi > 0
                if pi == len(passes) - 1 and exchanged:
                    chunks = [(c * GR, (c + 1) * GR) for c in range(G)]
                    split = h == 0 and X0.is_cuda and not self.host_staging
                    hub_done = (self._hub_first(csr, src[:, :W], dst[:, :W], chunks, h, own)
                                if split else [None] * G)
                    for c, rows in enumerate(chunks):  # final pass in row chunks, each sent at once
                        self.spmm_fn(csr, src[:, :W], dst[:, :W], rows, acc,
                                     "light" if split else "all", self._th, own=own)
                        new_works.append(self._issue(full[c * PGR:(c + 1) * PGR],
                                                     dst[c * GR:(c + 1) * GR], (h, c), hub_done[c]))
                else:
                    self.spmm_fn(csr, src[:, :W], dst[:, :W], (0, R), acc, "all", self._th,
                                 own=own)
            if exchanged:
                works, src, src_own = new_works, full, True
            else:
                return dst[:s.n_valid]
        for w in works:
            if w is not None:
                w.wait()
        if out is None:
            out = torch.empty((n, F), dtype=torch.float32, device=X0.device)
        P, Tg, b = s.world_size, s.rounds_per_group, s.tile
        # exchange layout (g, q, t', i) -> global order (g, t', q, i)
        glob = src.view(G, P, Tg, b, Fp).permute(0, 2, 1, 3, 4).reshape(G * Tg * P * b, Fp)
        out.copy_(glob[:n, :F])
        return out


# ---------------------------------------------------------------------------
# 2-D partition: row blocks x feature blocks.

class TiledPropagator:
    """X_K = S^K X_0 over P = R x C ranks: rank p = i*C + j owns row block i
    (nnz-balanced over R) of feature block j (C equal,
    4-aligned column blocks).  Each column block is an independent row
    partition over its R ranks (RowPartitionedPropagator on the sub-group of
    ranks holding block j): the all-gather between hops moves N x F/C floats
    per rank instead of N x F, and each rank's launches cover N/R rows
    instead of N/P, so every X line it gathers is reused by R/P-times more
    rows than under a pure row partition.  The row partition is C = 1.
    Bit-exact: each element is still one FMA chain over its row in CSR order.

    output="sharded": this rank's full-width row block [rows_i, F], assembled
    by one all-gather of the C tiles within the row group (ranks holding
    block i); output="tile": just the [rows_i, F/C] tile.

    Every rank must construct it collectively (it creates the sub-groups)."""

    def __init__(self, row_ptr, col_idx, val, rank, world_size, col_blocks, device,
                 group_floats=0, host_staging=False, balance="nnz", spmm_fn=None):
        C = int(col_blocks)
        if C < 1 or world_size % C:
            raise ValueError(f"col_blocks={C} must divide world_size={world_size}")
        R = world_size // C
        self.R, self.C = R, C
        self.i, self.j = rank // C, rank % C
        self.rank, self.world_size = rank, world_size
        self.host_staging = host_staging
        # every rank creates every sub-group, in the same order
        col_groups = [dist.new_group([i * C + j for i in range(R)]) for j in range(C)]
        row_groups = [dist.new_group([i * C + j for j in range(C)]) for i in range(R)]
        self.col_group, self.row_group = col_groups[self.j], row_groups[self.i]
        self.shard = make_shard(row_ptr, col_idx, val, self.i, R, device, balance=balance)
        self.prop = RowPartitionedPropagator(self.shard, group=self.col_group, spmm_fn=spmm_fn,
                                             group_floats=group_floats,
                                             host_staging=host_staging)
        self._bufs = {}

    @property
    def row_begin(self):
        return self.shard.row_begin

    @property
    def row_end(self):
        return self.shard.row_end

    def _buf(self, key, shape, like):
        b = self._bufs.get(key)
        if b is None or tuple(b.shape) != tuple(shape) or b.device != like.device:
            b = torch.empty(shape, dtype=torch.float32, device=like.device)
            self._bufs[key] = b
        return b

    def propagate(self, X0, K, out=None, output="sharded"):
        if output not in ("sharded", "tile"):
            raise ValueError(f"TiledPropagator output must be 'sharded' or 'tile', not {output!r}")
        n, F = X0.shape
        fb, Bf = feature_bounds(F, self.C)
        c0, c1 = int(fb[self.j]), int(fb[self.j + 1])
        rows = self.shard.rows
        if K <= 0:
            blk = X0[self.row_begin:self.row_end]
            return blk if output == "sharded" else blk[:, c0:c1]
        if self.C == 1:
            return self.prop.propagate(X0, K, out=out, output="sharded")
        tile = self._buf("tile", (max(1, rows), Bf), X0)[:rows]
        if c1 > c0:
            self.prop.propagate(X0[:, c0:c1], K, out=tile[:, :c1 - c0], output="sharded")
        if output == "tile":
            return tile[:, :c1 - c0]
        full = self._buf("tiles", (self.C * max(1, rows), Bf), X0)
        if self.host_staging:
            h = torch.empty(full.shape, dtype=full.dtype)
            dist.all_gather_into_tensor(h, self._buf("tile", (max(1, rows), Bf), X0).cpu(),
                                        group=self.row_group)
            full.copy_(h)
        else:
            dist.all_gather_into_tensor(full, self._buf("tile", (max(1, rows), Bf), X0),
                                        group=self.row_group)
        if out is None:
            out = torch.empty((rows, F), dtype=torch.float32, device=X0.device)
        R1 = max(1, rows)
        _copy_blocks(full, out, [(q * R1, 0, 0, int(fb[q]), rows, int(fb[q + 1] - fb[q]))
                                 for q in range(self.C)])
        return out


# ---------------------------------------------------------------------------
# Feature (column) partition.

def feature_bounds(F, world_size, align=4):
    """Column boundaries c_0=0 <= ... <= c_P=F: equal blocks of B floats, B =
    ceil(F/P) rounded up to `align` (so every block starts 16-B aligned and the
    SpMM can use its widest vector loads); the last blocks may be short or
    empty.  Returns (bounds [P+1], B)."""
    B = max(1, -(-F // world_size))
    B = -(-B // align) * align
    return np.minimum(np.arange(world_size + 1, dtype=np.int64) * B, F), B


def row_chunks(n, chunks):
    """[(r0, r1)] equal row ranges covering [0, n) (at most `chunks` of them)."""
    chunks = max(1, min(int(chunks), max(1, n)))
    step = -(-n // chunks) if n else 1
    return [(r, min(n, r + step)) for r in range(0, n, step)] or [(0, 0)]


def _copy_cols(src, dst):
    """dst[:, :] = src[:, :] for 2-D views with unit column stride: the HIP
    row-copy kernel on the GPU (the runtime's strided 2-D copy is ~3 TB/s on
    these shapes), torch on the CPU (the gloo rehearsal)."""
    if dst.numel() == 0:
        return
    if src.is_cuda:
        from . import _lib
        _lib.check(_lib.load().sgc_pad_rows_f32(
            _lib.ptr(src), src.stride(0), _lib.ptr(dst), dst.stride(0), dst.shape[0],
            dst.shape[1], _lib.stream_handle(src.device)), "pad_rows_f32")
    else:
        dst.copy_(src)


def _copy_blocks(src, dst, segs):
    """For (src_row, src_col, dst_row, dst_col, rows, cols) in segs:
    dst[dst_row:+rows, dst_col:+cols] = src[src_row:+rows, src_col:+cols], for
    2-D views with unit column stride: one sgc_copy_blocks_f32 launch per 64
    segments on the GPU (the exchanges' unpack: every rank's block of a
    gathered chunk at once), torch copies on the CPU."""
    segs = [tuple(int(v) for v in sg) for sg in segs if sg[4] > 0 and sg[5] > 0]
    if not segs:
        return
    if not src.is_cuda:
        for sr, sc, dr, dc, r, c in segs:
            dst[dr:dr + r, dc:dc + c].copy_(src[sr:sr + r, sc:sc + c])
        return
    import ctypes
    from . import _lib
    lib = _lib.load()
    for i in range(0, len(segs), 64):
        part = segs[i:i + 64]
        arr = (ctypes.c_int64 * (6 * len(part)))(*[v for sg in part for v in sg])
        _lib.check(lib.sgc_copy_blocks_f32(_lib.ptr(src), src.stride(0), _lib.ptr(dst),
                                           dst.stride(0), len(part), arr,
                                           _lib.stream_handle(src.device)), "copy_blocks_f32")


# Row fractions of the replicated output's last-hop chunks: a small first
# chunk (its all-gather starts as early as possible: at P = 8 the link time,
# not the hop, is the critical path), two large ones, a small last one (the
# last gather and unpack after the hop are short).  Measured against
# 1:1:2:3:1, 1:2:2:2:1, 1:2:3:2 (the same within noise at P = 8 and 4) and
# eight equal chunks (P = 8 2.71x vs 2.96x, P = 4 1.92x vs 1.88x),
# profiles/r05/rehearsal_fractions.log.
REPLICATED_CHUNKS = (1, 3, 3, 1)


def replicated_chunks(n, fractions=REPLICATED_CHUNKS):
    """[(r0, r1)] row ranges covering [0, n) in proportion to `fractions`
    (empty ranges dropped)."""
    tot = sum(fractions)
    cuts, acc = [0], 0
    for f in fractions:
        acc += f
        cuts.append(n * acc // tot)
    return [(a, b) for a, b in zip(cuts[:-1], cuts[1:]) if b > a] or [(0, n)]


def _chunk_order(csr, chunks):
    """Processing (and gathering) order of the last hop's row chunks: the
    chunk holding the graph's longest row last -- its hub chain (0.28 ms for
    Reddit shape's 47,857-nonzero row) delays that chunk, and with it last the
    link is kept busy with the others' gathers meanwhile.  Every rank
    computes all rows of its columns, so the order is the same on every rank
    (the collectives stay matched).  Natural order without a DeviceCSR."""
    if csr is None or not hasattr(csr, "row_ptr") or len(chunks) < 2:
        return list(range(len(chunks)))
    key = ("chunk_order", tuple(chunks))
    order = csr._plans.get(key)
    if order is None:
        # each chunk's longest row, on the adjacency's device (len(chunks)
        # ints come back, not the row_ptr)
        deg = csr.row_ptr[1:] - csr.row_ptr[:-1]
        longest = torch.stack([deg[r0:r1].max() if r1 > r0 else deg.new_zeros(())
                               for r0, r1 in chunks]).cpu().tolist()
        hub = int(np.argmax(longest))
        order = csr._plans[key] = [c for c in range(len(chunks)) if c != hub] + [hub]
    return order


# Schedule of the replicated last hop's chunks (A/B knobs of
# scripts/replicated_rehearsal.py; results never depend on them):
#  FIRST_CHUNK_ALONE  with CHUNK_STREAMS > 1: the other chunks start after
#                     the first one, so its gather (the link's first work) is
#                     not slowed by the chunk beside it (on one stream every
#                     chunk runs alone anyway);
#  HUB_EARLY          the hub rows of the chunk holding the longest row run
#                     early, on a stream of their own (with FIRST_CHUNK_ALONE:
#                     from the first chunk's end on, beside the chunks after
#                     it; else from the start), the rest of that chunk in its
#                     turn -- its serial chain no longer starts only when the
#                     chunks before it are done.  Launched at the start it
#                     delayed the first chunk by ~0.25 ms and every P=8
#                     projection dropped (profiles/r05/rehearsal_sched.log).
FIRST_CHUNK_ALONE = True
HUB_EARLY = False
# CHUNK_STREAMS      the chunks alternate between this many streams; 1 (in
#                     order on one stream, each chunk alone on the GPU, so its
#                     gather starts as early as it can): P = 8 lines 3.03x vs
#                     2.95-3.00x on two (profiles/r05/rehearsal_streams.log).
CHUNK_STREAMS = 1


def _replicated_last_hop(prop, n, P, p, ld, X0, hop_into, gather, unpack):
    """The replicated output's last hop (feature and line partitions): in row
    chunks (replicated_chunks), each computed into this rank's slot of its
    chunk's [P*rows, ld] gather buffer and all-gathered in place as soon as it
    is done; on the GPU the chunks run in order on one stream
    (CHUNK_STREAMS; with two, the first alone and the others alternating, a
    chunk's launch would not wait for the previous chunk's hub rows to join --
    measured slower); with HUB_EARLY the hub rows of the chunk
    holding the longest row (the last one, _chunk_order) start at once on a
    third stream (measured slower: they delay the first chunk).
    Each gather is issued from its chunk's stream and waits for exactly that
    chunk.  The caller's stream then waits for each gather and unpacks that
    chunk into X_K (one block-copy launch).
    hop_into(r0, r1, loc, flags=0) computes rows [r0, r1) into loc (flags:
    SPMM_HUB_ONLY / SPMM_NO_HUB for the split hub chunk); gather(full, loc)
    returns a work handle (or None: done on the current stream);
    unpack(full, r0, r1) lands the gathered chunk."""
    from .propagate import SPMM_HUB_ONLY, SPMM_NO_HUB
    gpu = X0.is_cuda
    if gpu:
        cur = torch.cuda.current_stream(X0.device)
        if getattr(prop, "_chunk_streams", None) is None or \
                prop._chunk_streams[0].device != X0.device:
            prop._chunk_streams = [torch.cuda.Stream(X0.device) for _ in range(3)]
    pending = []
    chunks = replicated_chunks(n, REPLICATED_CHUNKS if prop.chunks == 4 else (1,) * prop.chunks)
    order = _chunk_order(getattr(prop, "csr", None), chunks)
    hub_split = gpu and HUB_EARLY and len(order) > 1

    def hub_rows_first(after):
        # the hub chunk's hub rows, on a stream of their own from `after` on
        sh = prop._chunk_streams[2]
        if isinstance(after, torch.cuda.Event):
            sh.wait_event(after)
        else:
            sh.wait_stream(after)
        r0, r1 = chunks[order[-1]]
        full = prop._buf(("full", order[-1]), (P * (r1 - r0), ld), X0)
        with torch.cuda.stream(sh):
            hop_into(r0, r1, _gather_slot(full, p, r1 - r0), SPMM_HUB_ONLY)
    if hub_split and not FIRST_CHUNK_ALONE:
        hub_rows_first(cur)
    first_done = None
    for i, ci in enumerate(order):
        r0, r1 = chunks[ci]
        rows = r1 - r0
        full = prop._buf(("full", ci), (P * rows, ld), X0)
        loc = _gather_slot(full, p, rows)  # in-place gather: no copy of our block
        if gpu:
            st = prop._chunk_streams[i % CHUNK_STREAMS]
            st.wait_stream(cur)
            if first_done is not None and i % CHUNK_STREAMS:
                st.wait_event(first_done)
            split = hub_split and i == len(order) - 1
            with torch.cuda.stream(st):
                hop_into(r0, r1, loc, SPMM_NO_HUB if split else 0)
                if i == 0 and FIRST_CHUNK_ALONE:
                    first_done = torch.cuda.Event()
                    first_done.record(st)
                    if hub_split:  # beside the chunks after the first
                        hub_rows_first(first_done)
                if split:
                    st.wait_stream(prop._chunk_streams[2])
                work = gather(full, loc)
                if work is None:
                    work = _StreamDone(st)
        else:
            hop_into(r0, r1, loc)
            work = gather(full, loc)
        pending.append((r0, r1, full, work))
    for r0, r1, full, work in pending:
        if work is not None:
            work.wait()  # the caller's stream waits for this chunk's gather
        unpack(full, r0, r1)


# ---------------------------------------------------------------------------
# The replicated last hop over IPC-mapped peer memory (no gathered copy).

IPC_TIMEOUT_US = 20_000_000  # a peer silent this long: the call raises
IPC_FLAG_WORDS = 64          # int32 flags after the two halves: chunk c ready = word c,
IPC_DONE = 32                # this rank's pulls of a call done = word 32
IPC_TEST = 40                # the set-up self-test's flag


def replicated_exchange_mode(X0, world, force=False):
    """How the feature / line partitions hand out the replicated X_K:
    "ipc" (peers' blocks pulled straight into X_K's columns) on the GPU with
    more than one rank, else "collective" (in-place all-gather + unpack);
    SGC_AMD_REPLICATED_EXCHANGE=ipc|collective forces one."""
    import os
    m = os.environ.get("SGC_AMD_REPLICATED_EXCHANGE", "auto")
    if m not in ("auto", "ipc", "collective"):
        raise ValueError("SGC_AMD_REPLICATED_EXCHANGE must be auto, ipc or collective, "
                         f"not {m!r}")
    if not X0.is_cuda:
        return "collective"
    if m == "auto":
        return "ipc" if (world > 1 or force) else "collective"
    return m


class IpcPeers:
    """One rank's window for the replicated last hop, mapped by every peer.

    The window is one allocation: two [n, ld] fp32 halves (call s writes half
    s & 1, so a slow peer still reading call s-1's blocks is never
    overwritten; before writing half h again a rank waits for every peer's
    `done` flag of call s-2) and IPC_FLAG_WORDS int32 flags.  The handles are
    exchanged once through the process group (all_gather_object: gloo or
    RCCL), each peer's window opened with sgc_ipc_open (hipIpcOpenMemHandle:
    another GPU over xGMI, or the same GPU from another process in the
    one-GPU rehearsal).  `err` is a pinned host word the wait kernels set when
    a peer stays silent for IPC_TIMEOUT_US."""

    def __init__(self, group, rank, world, n, ld, device):
        import ctypes
        from . import _lib
        lib = _lib.load()
        self.rank, self.world, self.n, self.ld = rank, world, int(n), int(ld)
        self.ptrs, self._bases = [], []
        half = self.n * self.ld
        mine, why = None, ""
        try:
            self.window = torch.empty(2 * half + IPC_FLAG_WORDS, dtype=torch.float32,
                                      device=device)
            self.flags = self.window[2 * half:].view(torch.int32)
            self.flags.zero_()
            self.halves = [self.window[:half].view(self.n, self.ld),
                           self.window[half:2 * half].view(self.n, self.ld)]
            self.err = torch.zeros(1, dtype=torch.int32).pin_memory()
            torch.cuda.synchronize(device)  # zeroed flags before any peer reads them
            h = ctypes.create_string_buffer(128)
            if lib.sgc_ipc_get_handle(_lib.ptr(self.window), h) == 0:
                mine = h.raw
            else:
                why = lib.sgc_last_error().decode(errors="replace")
        except Exception as e:  # noqa: BLE001 -- reported after the exchange
            why = f"{type(e).__name__}: {e}"
        # every rank takes part in the exchange, whatever its own outcome (a
        # rank raising before it would leave the others in the collective)
        handles = [None] * world
        dist.all_gather_object(handles, mine, group=group)
        if any(x is None for x in handles):
            raise RuntimeError("sgc_amd: a rank could not export its IPC window" +
                               (f": {why}" if why else ""))
        try:
            for q in range(world):
                if q == rank:
                    self.ptrs.append(self.window.data_ptr())
                    continue
                base, ptr = ctypes.c_void_p(), ctypes.c_void_p()
                buf = ctypes.create_string_buffer(handles[q], 128)
                with torch.cuda.device(device):
                    _lib.check(lib.sgc_ipc_open(buf, ctypes.byref(base), ctypes.byref(ptr)),
                               "ipc_open")
                self._bases.append(base.value)
                self.ptrs.append(ptr.value)
        except Exception:
            self.close()
            raise
        self.seq = 0

    def half_ptr(self, q, h, row=0):
        return self.ptrs[q] + 4 * (h * self.n * self.ld + row * self.ld)

    def flag_ptr(self, q, word):
        return self.ptrs[q] + 4 * (2 * self.n * self.ld + word)

    def close(self):
        from . import _lib
        for b in self._bases:
            try:
                _lib.load().sgc_ipc_close(b)
            except Exception:  # interpreter shutdown
                pass
        self._bases = []

    def __del__(self):
        self.close()

    def signal(self, word, value, stream):
        from . import _lib
        _lib.check(_lib.load().sgc_signal_flag_i32(
            ctypes_void(self.flag_ptr(self.rank, word)), int(value),
            ctypes_void(stream.cuda_stream)), "signal_flag_i32")

    def wait(self, word, value, stream, ranks=None, timeout_us=IPC_TIMEOUT_US):
        import ctypes
        from . import _lib
        ranks = range(self.world) if ranks is None else list(ranks)
        ptrs = [self.flag_ptr(q, word) for q in ranks]
        if not ptrs:
            return
        arr = (ctypes.c_int64 * len(ptrs))(*ptrs)
        _lib.check(_lib.load().sgc_wait_flags_i32(len(ptrs), arr, int(value),
                                                  ctypes_void(self.err.data_ptr()),
                                                  int(timeout_us),
                                                  ctypes_void(stream.cuda_stream)),
                   "wait_flags_i32")

    def self_test(self, timeout_us=5_000_000):
        """Once, after mapping: every rank writes rank + 1 into the first row
        of its half 0 and raises flag IPC_TEST; every rank waits for its
        peers' flags and pulls their first rows.  True when each pulled value
        is its peer's rank + 1 -- the mapping, the flags' visibility and the
        pulls work between these processes (and GPUs); else the group keeps
        the collective path (a wrong byte would otherwise reach X_K)."""
        import ctypes
        from . import _lib
        stream = torch.cuda.current_stream(self.window.device)
        w = max(1, min(self.ld, 64))
        self.halves[0][0, :w].fill_(float(self.rank + 1))
        self.signal(IPC_TEST, 1, stream)
        self.wait(IPC_TEST, 1, stream, ranks=[q for q in range(self.world) if q != self.rank],
                  timeout_us=timeout_us)
        got = torch.zeros((1, w * self.world), dtype=torch.float32, device=self.window.device)
        segs = [(self.half_ptr(q, 0, 0), self.ld, 0, q * w, 1, w) for q in range(self.world)]
        for i in range(0, len(segs), 16):
            part = segs[i:i + 16]
            arr = (ctypes.c_int64 * (6 * len(part)))(*[v for sg in part for v in sg])
            _lib.check(_lib.load().sgc_pull_blocks_f32(len(part), arr, _lib.ptr(got), got.stride(0),
                                                       ctypes_void(stream.cuda_stream)),
                       "pull_blocks_f32")
        stream.synchronize()
        if int(self.err[0]) != 0:
            self.err.zero_()
            return False
        want = torch.arange(1, self.world + 1, dtype=torch.float32).repeat_interleave(w)
        return bool(torch.equal(got.cpu()[0], want))

    def check(self, stream):
        """After the caller's stream is done: raise if a wait timed out."""
        stream.synchronize()
        if int(self.err[0]) != 0:
            self.err.zero_()
            raise RuntimeError("sgc_amd: a peer's block of the replicated X_K never became "
                               f"ready within {IPC_TIMEOUT_US / 1e6:.0f} s (IPC exchange)")


def ctypes_void(v):
    import ctypes
    return ctypes.c_void_p(int(v))


# Host seconds of the set-up stages of the first partitioned call, by stage
# (measurement: with SGC_AMD_SETUP_TRACE=1 each stage also synchronises the
# device first, so the GPU work it queued is charged to it).
SETUP_SECONDS = {}


@contextlib.contextmanager
def setup_stage(name, device=None):
    if os.environ.get("SGC_AMD_SETUP_TRACE") != "1":
        yield
        return
    if device is not None and device.type == "cuda":
        torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    try:
        yield
    finally:
        if device is not None and device.type == "cuda":
            torch.cuda.synchronize(device)
        SETUP_SECONDS[name] = SETUP_SECONDS.get(name, 0.0) + time.perf_counter() - t0


def _ipc_for(prop, group, rank, world, n, ld, device):
    """The propagator's IpcPeers window for [n, ld] halves, made once
    (collective: every rank builds it in the same call); None when a rank
    could not map its peers -- then every rank keeps the collective path."""
    key = (n, ld, str(device))
    if getattr(prop, "_ipc_key", None) == key:
        return prop._ipc
    ok, ipc, why = 1, None, ""
    try:
        with setup_stage("ipc_window_and_handles", device):
            ipc = IpcPeers(group, rank, world, n, ld, device)
        with setup_stage("ipc_self_test", device):
            passed = ipc.self_test()
        if not passed:
            ok, why = 0, "the set-up self-test read a wrong value or timed out"
    except Exception as e:  # noqa: BLE001 -- recorded, agreed on below
        ok, why = 0, f"{type(e).__name__}: {e}"
    if world > 1:
        with setup_stage("ipc_agree", device):
            dev = device if dist.get_backend(group) == "nccl" else torch.device("cpu")
            t = torch.tensor([ok], dtype=torch.int32, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
            ok = int(t.item())
    if not ok:
        if ipc is not None:
            ipc.close()
        ipc = None
        prop.ipc_unavailable = why or "a peer could not map the windows"
    prop._ipc, prop._ipc_key = ipc, key
    return ipc


def _replicated_last_hop_ipc(prop, ipc, n, P, p, X0, hop_into, blocks, out):
    """The replicated output's last hop through IpcPeers: the rows in the
    chunks and order of _replicated_last_hop, each computed into this rank's
    half of its window on the chunk stream and announced by a flag; the
    caller's stream then, per chunk, waits for its own event and every
    peer's flag and pulls all P column blocks (blocks[q] = (col0, width) of
    rank q in X_K) straight into `out` -- one sgc_pull_blocks_f32 launch per
    chunk, no gather buffer, no unpack.  Bit-identical: the bytes are moved,
    never recomputed."""
    import ctypes
    from . import _lib
    lib = _lib.load()
    ipc.seq += 1
    seq, h = ipc.seq, ipc.seq & 1
    mine = ipc.halves[h]
    cur = torch.cuda.current_stream(X0.device)
    if getattr(prop, "_chunk_streams", None) is None or \
            prop._chunk_streams[0].device != X0.device:
        prop._chunk_streams = [torch.cuda.Stream(X0.device) for _ in range(3)]
    st = prop._chunk_streams[0]
    st.wait_stream(cur)
    chunks = replicated_chunks(n, REPLICATED_CHUNKS if prop.chunks == 4 else (1,) * prop.chunks)
    order = _chunk_order(getattr(prop, "csr", None), chunks)
    if len(order) > 32:
        raise ValueError("IPC exchange: at most 32 chunks")
    evs = []
    with torch.cuda.stream(st):
        if seq > 2:  # every peer is done reading this half (call seq - 2)
            ipc.wait(IPC_DONE, seq - 2, st, ranks=[q for q in range(P) if q != p])
        for ci in order:
            r0, r1 = chunks[ci]
            hop_into(r0, r1, mine[r0:r1])
            ipc.signal(ci, seq, st)
            ev = torch.cuda.Event()
            ev.record(st)
            evs.append(ev)
    max_rows = max(1, ((1 << 31) - 1) // (4 * ipc.ld) - 1)  # a segment's span < 2 GiB
    for ci, ev in zip(order, evs):
        r0, r1 = chunks[ci]
        cur.wait_event(ev)
        ipc.wait(ci, seq, cur, ranks=[q for q in range(P) if q != p])
        segs = []
        for a in range(r0, r1, max_rows):
            b = min(r1, a + max_rows)
            for q in range(P):
                c0, w = blocks[q]
                if w > 0:
                    segs.append((ipc.half_ptr(q, h, a), ipc.ld, a, c0, b - a, w))
        for i in range(0, len(segs), 16):
            part = segs[i:i + 16]
            arr = (ctypes.c_int64 * (6 * len(part)))(*[v for sg in part for v in sg])
            _lib.check(lib.sgc_pull_blocks_f32(len(part), arr, _lib.ptr(out), out.stride(0),
                                               ctypes_void(cur.cuda_stream)), "pull_blocks_f32")
    ipc.signal(IPC_DONE, seq, cur)


def _gather_slot(full, p, rows):
    """Rank p's slot of an all-gather buffer [P*rows, ld]: the last hop writes
    its rows there and the gather runs in place (NCCL/RCCL in-place
    all-gather: sendbuff = recvbuff + rank*count), so the rank's own block is
    never copied."""
    return full[p * rows:(p + 1) * rows]


class FeaturePartitionedPropagator:
    """X_K = S^K X_0 with the feature columns split over the process group.

    Column f of X_{k+1} = S . column f of X_k, so a column block never needs
    another rank's data between hops: rank p copies its block [c_p, c_{p+1})
    of X_0 into a compact 128-B-row buffer (at P=8 and Reddit shape 233k x 76
    floats = 71 MB, resident in the 256 MB Infinity Cache, where the full
    561 MB X never is), runs the K hops over the full CSR (every rank holds all
    of S: 0.19 GB at Reddit shape), and the only exchange is one all-gather of
    the column blocks of X_K -- half the bytes the row partition moves at K=2
    (per-hop all-gather + final gather), a third at K=3.  The last hop runs in
    `chunks` row ranges; chunk c's all-gather (async, RCCL stream) overlaps the
    SpMM of chunk c+1, and each gathered chunk [P, rows, B] is unpacked into
    the [N, F] result once it has arrived.

    Every element is still the same single FMA chain in CSR order, so the
    result is bit-identical to one GPU's and to the reference.

    output="sharded" exchanges the row blocks of X_K either with one
    all-to-all after the last hop (exchange="alltoall") or pairwise, overlapped
    with the last hop (exchange="pairwise"): rank p computes the rows it owes
    rank p+1 first, then p+2, ..., its own rows last, and step j of the
    exchange (send to p+j, receive from p-j; both sides post the same (step,
    piece) sequence, so the P2P pairs match) is enqueued as soon as its rows
    are computed, in `pieces` row pieces per destination (default 4 at
    P = 2).  On xGMI every GPU pair has one link, so at P = 2 the
    all-to-all's 142 MB (Reddit shape)
    crosses ONE link after the last hop; pairwise, it rides under the
    computation of the rows that follow.  exchange="auto": pairwise at P = 2
    only.  Each destination piece is a launch of its own, and a split hop pays
    every launch's ramp-down tail: measured on one GPU per rank (Reddit shape,
    profiles/r03/s12/feat.log) the rank's compute grows 5.19 -> 5.74 ms at
    P = 2 (3 launches), 3.05 -> 3.43 at P = 4, 1.67 -> 2.41 at P = 8, so with
    one 57.6 GB/s link per GPU pair the projected step is 7.65 -> 6.38 ms at
    P = 2, 3.66 -> 3.69 at P = 4 and 1.83 -> 2.47 at P = 8 (with the column
    groups and 4 pieces at P = 2: 7.40 -> 6.08 ms, profiles/r03/s17/).

    spmm_fn(X, row_begin, row_end, out) computes rows [row_begin, row_end) of
    S.X for the columns X has; the default is the HIP kernel over the cached
    DeviceCSR (tests inject the CPU oracle to run the exchange over gloo)."""

    def __init__(self, csr=None, rank=None, world_size=None, group=None,
                 spmm_fn: Optional[Callable] = None, chunks: int = 4,
                 host_staging: bool = False, align: int = 4, exchange: str = "auto",
                 pieces: Optional[int] = None):
        if exchange not in ("auto", "alltoall", "pairwise"):
            raise ValueError(f"exchange must be 'auto', 'alltoall' or 'pairwise', not {exchange!r}")
        self.group = group
        self.rank = dist.get_rank(group) if rank is None else int(rank)
        self.world_size = dist.get_world_size(group) if world_size is None else int(world_size)
        self._padded_ok = spmm_fn is None  # the engine's own launches take pad flags
        if spmm_fn is None:
            if csr is None:
                raise ValueError("FeaturePartitionedPropagator needs a DeviceCSR or an spmm_fn")
            from .propagate import spmm

            def spmm_fn(X, r0, r1, out, flags=0, _csr=csr):
                return spmm(_csr, X, r0, r1, out=out, flags=flags)
        self.csr = csr
        self.spmm_fn = spmm_fn
        self.chunks = max(1, int(chunks))
        self.align = max(1, int(align))
        self.host_staging = host_staging  # rehearsal only: gathers through host copies (gloo)
        self.exchange = exchange
        self.pieces = pieces
        self._bufs = {}

    # test hook: run the exchange through the process group even at world 1
    # (the one-rank shortcuts skip it), so a one-GPU box exercises the RCCL
    # calls -- async all-gathers from a side stream, in-place slots, waits
    # across streams -- that P > 1 runs
    force_collectives = False
    # test hook: the replicated last hop through the IPC window at world 1
    # (its own block pulled by sgc_pull_blocks_f32, flags signalled/awaited)
    force_ipc = False
    ipc_unavailable = None  # why the IPC window could not be mapped, if so

    def _buf(self, key, shape, like):
        b = self._bufs.get(key)
        if b is None or tuple(b.shape) != tuple(shape) or b.device != like.device:
            b = torch.empty(shape, dtype=torch.float32, device=like.device)
            self._bufs[key] = b
        return b

    def _all_gather(self, full, loc):
        if not self.host_staging:
            return dist.all_gather_into_tensor(full, loc, group=self.group, async_op=True)
        h_full = torch.empty(full.shape, dtype=full.dtype)
        dist.all_gather_into_tensor(h_full, loc.cpu(), group=self.group)
        full.copy_(h_full)
        return None

    def _all_to_all(self, recv, send):
        if not self.host_staging:
            return dist.all_to_all_single(recv, send, group=self.group, async_op=True)
        h_recv = torch.empty(recv.shape, dtype=recv.dtype)
        dist.all_to_all_single(h_recv, send.cpu(), group=self.group)
        recv.copy_(h_recv)
        return None

    def _global(self, r):
        return r if self.group is None else dist.get_global_rank(self.group, r)

    def _exchange_pair(self, send, dst, recv, src):
        """One step of the pairwise exchange: send -> rank dst, recv <- rank
        src (group ranks; an empty side is skipped -- its partner computes the
        same empty range).  Returns the works to wait on (none when staged)."""
        staged = self.host_staging
        h_recv = torch.empty(recv.shape, dtype=recv.dtype) if staged else recv
        ops = []
        if send.numel():
            ops.append(dist.P2POp(dist.isend, send.cpu() if staged else send,
                                  self._global(dst), group=self.group))
        if recv.numel():
            ops.append(dist.P2POp(dist.irecv, h_recv, self._global(src), group=self.group))
        if not ops:
            return []
        works = dist.batch_isend_irecv(ops)
        if not staged:
            return works
        for w_ in works:
            w_.wait()
        recv.copy_(h_recv)
        return []

    def _pieces(self, P):
        if self.pieces is not None:
            return max(1, int(self.pieces))
        # P = 2 over one link: 4 pieces per destination (projected, one GPU per
        # rank: 6.65 / 6.40 / 6.16 / 6.08 / 6.34 ms at 1 / 2 / 3 / 4 / 6 pieces,
        # profiles/r03/s17/feat_p2_pieces*.log)
        return 4 if P == 2 else 1

    def _sharded_pairwise(self, src, own, out, hop, bounds, B, rb, X0):
        """Last hop + pairwise exchange of the row blocks (class docstring)."""
        n = X0.shape[0]
        P, p = self.world_size, self.rank
        c0, c1 = int(bounds[p]), int(bounds[p + 1])
        w = c1 - c0
        Bn = max(1, -(-n // P))
        send = self._buf("send", (P * Bn, B), X0)
        recv = self._buf("recv", (P * Bn, B), X0)
        k = self._pieces(P)
        mine0, mine1 = int(rb[p]), int(rb[p + 1])
        works = []
        for j in range(1, P):
            q, s_ = (p + j) % P, (p - j) % P
            q0, q1 = int(rb[q]), int(rb[q + 1])
            for i in range(k):  # exactly k pieces on both sides (some may be empty)
                a, b = (q1 - q0) * i // k, (q1 - q0) * (i + 1) // k
                ra, rb_ = (mine1 - mine0) * i // k, (mine1 - mine0) * (i + 1) // k
                if w and b > a:  # send's columns w..B-1 are never unpacked: pad-writable
                    hop(src, q0 + a, q0 + b, send[q0 + a:q0 + b, :w], own, True)
                works += self._exchange_pair(send[q0 + a:q0 + b], q,
                                             recv[s_ * Bn + ra:s_ * Bn + rb_], s_)
        if w and mine1 > mine0:  # own rows straight into the result
            hop(src, mine0, mine1, out[:, c0:c1], own, False)
        for w_ in works:
            w_.wait()
        rows = mine1 - mine0
        _copy_blocks(recv, out, [(s_ * Bn, 0, 0, int(bounds[s_]), rows,
                                  int(bounds[s_ + 1] - bounds[s_])) for s_ in range(P) if s_ != p])
        return out

    def propagate(self, X0, K, out=None, output="replicated"):
        """output="replicated": the full X_K on every rank (one all-gather).
        output="sharded": this rank's rows [r_p, r_{p+1}) of X_K (equal-row
        blocks, equal_row_bounds) as a [rows, F] tensor: the last hop is
        computed per destination row block and the blocks are exchanged by one
        all-to-all (1/P of the all-gather's bytes)."""
        if output not in ("replicated", "sharded"):
            raise ValueError(f"output must be 'replicated' or 'sharded', not {output!r}")
        n, F = X0.shape
        P, p = self.world_size, self.rank
        rb = equal_row_bounds(n, P)
        if K <= 0:
            return X0 if output == "replicated" else X0[int(rb[p]):int(rb[p + 1])]
        bounds, B = feature_bounds(F, P, self.align)
        c0, c1 = int(bounds[p]), int(bounds[p + 1])
        w = c1 - c0
        ld = (B + 31) // 32 * 32 if X0.is_cuda else B  # 128-B rows on the GPU
        if out is None:
            shape = (n, F) if output == "replicated" else (int(rb[p + 1] - rb[p]), F)
            out = torch.empty(shape, dtype=torch.float32, device=X0.device)
        from .propagate import SPMM_X_PADDED, SPMM_Y_PADDED

        def hop(src, r0, r1, dst, own_src, own_dst, flags=0):
            # own buffers: 4-float pad columns may be read / written (16-B
            # lanes at any block width); results never depend on it
            if self._padded_ok:
                flags |= (SPMM_X_PADDED if own_src else 0) | (SPMM_Y_PADDED if own_dst else 0)
            if flags:
                return self.spmm_fn(src, r0, r1, dst, flags=flags)
            return self.spmm_fn(src, r0, r1, dst)

        # hop 1 reads the caller's block in place when its rows are 16-B
        # lanes already (w and c0 multiples of 4, 16-B aligned rows); else a
        # compact 128-B-row copy first
        inplace = (K == 1 or not X0.is_cuda or
                   (w % 4 == 0 and c0 % 4 == 0 and X0.stride(0) % 4 == 0 and
                    X0.data_ptr() % 16 == 0))
        src, own = X0[:, c0:c1], False
        if not inplace:
            a = self._buf("a", (n, ld), X0)
            _copy_cols(X0[:, c0:c1], a[:, :w])
            src, own = a[:, :w], True
        # hops 1..K-1 on the rank's column block, ping-pong in compact buffers
        for h in range(K - 1):
            dst = self._buf(("h", h & 1), (n, ld), X0)[:, :w]
            if w and n:
                hop(src, 0, n, dst, own, True)
            src, own = dst, True
        if P == 1 and not (self.force_collectives or self.force_ipc):
            if w and n:  # the last hop writes X_K itself
                hop(src, 0, n, out, own, False)
            return out
        if output == "sharded" and (self.exchange == "pairwise" or
                                    (self.exchange == "auto" and P == 2)):
            return self._sharded_pairwise(src, own, out, hop, bounds, B, rb, X0)
        if output == "sharded":
            # last hop -> one all-to-all.  Destination block q is rows
            # [q*Bn, (q+1)*Bn) (equal_row_bounds), so ONE launch over all rows
            # into send[:n] already lays the send buffer out by destination
            # (a launch per block would pay the hub fork/join P times)
            Bn = max(1, -(-n // P))
            send = self._buf("send", (P * Bn, B), X0)
            if w and n:  # send's columns w..B-1 are never unpacked: pad-writable
                hop(src, 0, n, send[:n, :w], own, True)
            recv = self._buf("recv", (P * Bn, B), X0)
            work = self._all_to_all(recv, send)
            if work is not None:
                work.wait()
            rows = int(rb[p + 1] - rb[p])
            _copy_blocks(recv, out, [(q * Bn, 0, 0, int(bounds[q]), rows,
                                      int(bounds[q + 1] - bounds[q])) for q in range(P)])
            return out
        # last hop in row chunks, each computed into this rank's slot of the
        # chunk's gather buffer and gathered in place as soon as it is done;
        # every gathered chunk then lands in X_K's columns in one launch

        def hop_into(r0, r1, loc, flags=0):
            if w:
                hop(src, r0, r1, loc[:, :w], own, True, flags)

        if replicated_exchange_mode(X0, P, self.force_ipc) == "ipc":
            ipc = _ipc_for(self, self.group, p, P, n, ld, X0.device)
            if ipc is not None:
                blocks = [(int(bounds[q]), int(bounds[q + 1] - bounds[q])) for q in range(P)]
                _replicated_last_hop_ipc(self, ipc, n, P, p, X0, hop_into, blocks, out)
                ipc.check(torch.cuda.current_stream(X0.device))
                return out

        def unpack(full, r0, r1):
            rows = r1 - r0
            _copy_blocks(full, out, [(q * rows, 0, r0, int(bounds[q]), rows,
                                      int(bounds[q + 1] - bounds[q])) for q in range(P)])
        _replicated_last_hop(self, n, P, p, B, X0, hop_into, self._all_gather, unpack)
        return out


# ---------------------------------------------------------------------------
# Line partition: whole 128-B lines of features per rank + a row-sharded tail.

def line_bounds(F, world_size, line=32):
    """Feature layout of the line partition: every rank owns W = m*line
    columns (m = ceil(F/line) // P whole 128-B lines) -- main block p is
    [min(p*W, F), min((p+1)*W, F)) -- and the tail [T, F), T = min(P*W, F),
    is computed by row blocks.  Returns (W, T)."""
    lines = -(-F // line)
    W = (lines // world_size) * line
    return W, min(F, world_size * W)


class LinePartitionedPropagator:
    """X_K = S^K X_0 with each rank owning whole 128-B lines of features plus
    a row block of the leftover (tail) features.

    What a hop costs on the GPU follows the 128-B lines each gathered row
    segment touches: one GPU gathers ceil(F/32) lines per
    nonzero (19 at F = 602); the feature partition's 76-float blocks gather 3
    per nonzero on EVERY rank at P = 8 (24 in all), 152-float blocks 5 at
    P = 4 (20).  Here rank p gathers m = ceil(F/32) // P whole lines over all
    rows -- main block [p*W, (p+1)*W), W = 32m floats, no exchange between
    hops, as in the feature partition -- and the tail's L - P*m lines (3 at F =
    602 for P = 4 and 8) over its nnz-balanced row block only, so every rank
    gathers m + (L - P*m)/P lines per nonzero: 2.375 at P = 8, 4.75 at P = 4.
    The tail's row blocks are all-gathered after each hop into the [P*B, wt]
    exchange buffer (B = the largest block) that the next hop's tail launch
    reads through the shard's gathered column ids (RowPartitionedPropagator's
    layout).  On the GPU the tail launches and their gathers run on a stream
    of their own beside the main launches: a tail launch is small (1/P of
    the nonzeros) and pays its ramp, its launch tail and its hub chains in
    full when it runs alone, and the gather of hop k then rides under main
    hop k as well.

    Every element is still one FMA chain in CSR order: bit-identical to one
    GPU and to the reference.

    output="replicated": every rank gets X_K (the main blocks of the last hop
    all-gathered in row chunks as they are computed, the tail from the last
    gather); output="sharded": rank p gets rows [r_p, r_{p+1}) of X_K
    (equal_row_bounds; the main blocks by one all-to-all).

    main_spmm_fn(X, r0, r1, out, flags=0) computes rows [r0, r1) of S.X over
    the full CSR (default: the HIP engine over `csr`); tail_spmm_fn(shard, X,
    out, layout) computes the shard's rows (default: _default_spmm).  Tests
    inject the CPU oracle for both."""

    def __init__(self, shard: ShardCSR, csr=None, group=None,
                 main_spmm_fn: Optional[Callable] = None,
                 tail_spmm_fn: Optional[Callable] = None, chunks: int = 4,
                 host_staging: bool = False):
        self.shard = shard
        self.group = group
        self.rank, self.world_size = shard.rank, shard.world_size
        self._padded_ok = main_spmm_fn is None
        if main_spmm_fn is None:
            if csr is None:
                raise ValueError("LinePartitionedPropagator needs a DeviceCSR or a main_spmm_fn")
            from .propagate import spmm

            def main_spmm_fn(X, r0, r1, out, flags=0, _csr=csr):
                return spmm(_csr, X, r0, r1, out=out, flags=flags)
        self.csr = csr  # (None with injected launches)
        self.main_spmm_fn = main_spmm_fn
        self.tail_spmm_fn = tail_spmm_fn or _default_spmm
        self.chunks = max(1, int(chunks))
        self.host_staging = host_staging
        self._bufs = {}
        self._tail_stream = None

    def _buf(self, key, shape, like):
        b = self._bufs.get(key)
        if b is None or tuple(b.shape) != tuple(shape) or b.device != like.device:
            b = torch.empty(shape, dtype=torch.float32, device=like.device)
            self._bufs[key] = b
        return b

    def _tail_ctx(self, device):
        """Context running the tail's launches and gathers on the tail stream
        (a no-op on the CPU)."""
        import contextlib
        if device.type != "cuda":
            return contextlib.nullcontext()
        if self._tail_stream is None or self._tail_stream.device != device:
            self._tail_stream = torch.cuda.Stream(device)
        return torch.cuda.stream(self._tail_stream)

    force_collectives = False  # test hooks, as FeaturePartitionedPropagator's
    force_ipc = False
    ipc_unavailable = None

    def _collective(self, kind, dst, src):
        if self.world_size == 1 and not self.force_collectives:
            return _local_copy(dst, src)
        fn = dist.all_gather_into_tensor if kind == "gather" else dist.all_to_all_single
        if not self.host_staging:
            return fn(dst, src, group=self.group, async_op=True)
        h = torch.empty(dst.shape, dtype=dst.dtype)
        fn(h, src.cpu(), group=self.group)
        dst.copy_(h)
        return None

    def _tail_rows(self, full, wt, r0, r1, dst):
        """dst[:] = tail rows [r0, r1) of the gathered [P*B, ld] buffer (they
        may span several ranks' blocks)."""
        sh = self.shard
        B = sh.block
        segs = []
        for q in range(self.world_size):
            a, b = max(r0, int(sh.bounds[q])), min(r1, int(sh.bounds[q + 1]))
            if b > a:
                segs.append((q * B + a - int(sh.bounds[q]), 0, a - r0, 0, b - a, wt))
        _copy_blocks(full, dst, segs)

    def propagate(self, X0, K, out=None, output="replicated"):
        if output not in ("replicated", "sharded"):
            raise ValueError(f"output must be 'replicated' or 'sharded', not {output!r}")
        n, F = X0.shape
        P, p = self.world_size, self.rank
        sh = self.shard
        if sh.n != n:
            raise ValueError(f"shard has {sh.n} nodes, features {n}")
        rb = equal_row_bounds(n, P)
        if K <= 0:
            return X0 if output == "replicated" else X0[int(rb[p]):int(rb[p + 1])]
        W, T = line_bounds(F, P)
        c0, c1 = min(p * W, F), min((p + 1) * W, F)
        w, wt = c1 - c0, F - T
        gpu = X0.is_cuda
        ld = (max(W, 1) + 31) // 32 * 32 if gpu else max(W, 1)
        ldt = (max(wt, 1) + 31) // 32 * 32 if gpu else max(wt, 1)
        if out is None:
            shape = (n, F) if output == "replicated" else (int(rb[p + 1] - rb[p]), F)
            out = torch.empty(shape, dtype=torch.float32, device=X0.device)
        from .propagate import SPMM_X_PADDED, SPMM_Y_PADDED

        def main_hop(src, r0, r1, dst, own_src, own_dst, flags=0):
            if self._padded_ok:
                flags |= (SPMM_X_PADDED if own_src else 0) | (SPMM_Y_PADDED if own_dst else 0)
            if flags:
                return self.main_spmm_fn(src, r0, r1, dst, flags=flags)
            return self.main_spmm_fn(src, r0, r1, dst)

        def aligned(v, col0, width):  # 16-B lanes readable in place
            return (not gpu or (width % 4 == 0 and col0 % 4 == 0 and v.stride(0) % 4 == 0 and
                                v.data_ptr() % 16 == 0))

        # hop-1 inputs: the rank's main block and the tail, in 128-B rows
        msrc, mown = X0[:, c0:c1], False
        if w and K > 1 and not aligned(X0, c0, w):
            a = self._buf("a", (n, ld), X0)
            _copy_cols(X0[:, c0:c1], a[:, :w])
            msrc, mown = a[:, :w], True
        # tail launches on the engine's own 128-B-row buffers compute wt
        # rounded up to 4 columns (16-B lanes; the pad columns are never read
        # back), on the caller's X_0 exactly wt
        wt4 = min(ldt, (wt + 3) // 4 * 4) if gpu else wt
        tsrc, tlayout, tw = X0[:, T:F], "input", wt
        if wt and gpu and not aligned(X0, T, wt):
            ta = self._buf("ta", (n, ldt), X0)
            _copy_cols(X0[:, T:F], ta[:, :wt])
            tsrc, tw = ta[:, :wt4], wt4
        B = sh.block
        work = None
        full = None
        if gpu and wt:  # the tail stream starts after the inputs (and last call)
            cur = torch.cuda.current_stream(X0.device)
            with self._tail_ctx(X0.device):
                torch.cuda.current_stream(X0.device).wait_stream(cur)
        for k in range(1, K + 1):
            # tail: this rank's rows of hop k, gathered at once for hop k+1
            if wt:
                with self._tail_ctx(X0.device):
                    if work is not None:
                        work.wait()
                    # this hop's gather buffer (hop k-1's is the one being
                    # read: two alternate); the tail launch writes our slot
                    # and the gather runs in place
                    full = self._buf(("tf", k & 1), (P * B, ldt), X0)
                    loc = _gather_slot(full, p, B)
                    if sh.rows:
                        self.tail_spmm_fn(sh, tsrc, loc[:sh.rows, :tw], tlayout)
                    work = self._collective("gather", full, loc)
                    if work is None and gpu:  # staged: the copy is done on this stream
                        work = _StreamDone(torch.cuda.current_stream(X0.device))
                tsrc, tlayout, tw = full[:, :wt4], "gathered", wt4
            # main block of hop k (no exchange between hops)
            if k < K:
                dst = self._buf(("h", k & 1), (n, ld), X0)[:, :w]
                if w and n:
                    main_hop(msrc, 0, n, dst, mown, True)
                msrc, mown = dst, True
                continue
            if output == "replicated":
                self._last_replicated(msrc, mown, out, main_hop, W, w, ld, P, X0)
            else:
                self._last_sharded(msrc, mown, out, main_hop, W, w, rb, P, X0)
        if work is not None:
            work.wait()
        if wt:  # the tail of X_K from the last gather
            r0, r1 = (0, n) if output == "replicated" else (int(rb[p]), int(rb[p + 1]))
            self._tail_rows(full, wt, r0, r1, out[:, T:F])
        ipc, self._ipc_pending = getattr(self, "_ipc_pending", None), None
        if ipc is not None:
            ipc.check(torch.cuda.current_stream(X0.device))
        return out

    def _last_replicated(self, msrc, mown, out, main_hop, W, w, ld, P, X0):
        n, F = out.shape
        if P == 1 and not (self.force_collectives or self.force_ipc):
            if w and n:
                main_hop(msrc, 0, n, out[:, :w], mown, False)
            return
        if W == 0:  # all-tail layout (F < 32 P): no main blocks to exchange (W is
            return  # the same on every rank, so every rank skips the same calls)
        def hop_into(r0, r1, loc, flags=0):
            if w:
                main_hop(msrc, r0, r1, loc[:, :w], mown, True, flags)

        if replicated_exchange_mode(X0, P, self.force_ipc) == "ipc":
            ipc = _ipc_for(self, self.group, self.rank, P, n, ld, X0.device)
            if ipc is not None:
                blocks = [(min(q * W, F), min((q + 1) * W, F) - min(q * W, F)) for q in range(P)]
                _replicated_last_hop_ipc(self, ipc, n, P, self.rank, X0, hop_into, blocks, out)
                self._ipc_pending = ipc
                return

        def unpack(full, r0, r1):
            rows = r1 - r0
            _copy_blocks(full, out, [(q * rows, 0, r0, min(q * W, F), rows,
                                      min((q + 1) * W, F) - min(q * W, F)) for q in range(P)])
        _replicated_last_hop(self, n, P, self.rank, ld, X0, hop_into,
                             lambda full, loc: self._collective("gather", full, loc), unpack)

    def _last_sharded(self, msrc, mown, out, main_hop, W, w, rb, P, X0):
        n = msrc.shape[0]
        F = out.shape[1]
        p = self.rank
        if W == 0:  # all-tail layout: nothing in the main blocks (same on every rank)
            return
        Bn = max(1, -(-n // P))
        ldw = max(W, 1)
        send = self._buf("send", (P * Bn, ldw), X0)
        if w and n:
            main_hop(msrc, 0, n, send[:n, :w], mown, True)
        recv = self._buf("recv", (P * Bn, ldw), X0)
        work = self._collective("a2a", recv, send)
        if work is not None:
            work.wait()
        rows = int(rb[p + 1] - rb[p])
        _copy_blocks(recv, out, [(q * Bn, 0, 0, min(q * W, F), rows,
                                  min((q + 1) * W, F) - min(q * W, F)) for q in range(P)])


# ---------------------------------------------------------------------------
# Data-parallel classifier over a row-sharded X_K.

def _torch_loss_grad(X, W, b, y):
    """(mean loss, dW, db) of F.cross_entropy(X W^T + b, y) by torch autograd
    (the CPU rehearsal's stand-in for the fused HIP kernel)."""
    W_ = W.detach().clone().requires_grad_(True)
    b_ = None if b is None else b.detach().clone().requires_grad_(True)
    z = X @ W_.t() + (b_ if b_ is not None else 0)
    loss = torch.nn.functional.cross_entropy(z, y)
    loss.backward()
    return loss.detach(), W_.grad, (None if b_ is None else b_.grad)


class ShardedSGCTrainer:
    """Trains the SGC classifier (models.SGC: logits = X W^T + b) data-parallel
    over the row blocks the propagators return with output="sharded".

    Reference: the training closures of reddit.py:51-64 (LBFGS) and
    citation.py:35-58 (Adam) compute F.cross_entropy(model(X[idx]), y[idx])
    over all training rows.  Here each rank holds the training rows inside its
    own row block; `loss()` computes the rank's loss and gradients in one fused
    pass (sgc_linear_xent_f32: GEMM + softmax-CE forward + dW/db), scales them
    by m_rank / M, and one all-reduce of [loss, dW, db] (4 + 4C(F+1) bytes:
    ~99 KB at Reddit shape) gives every rank the global mean loss and
    gradients, which it writes into the parameters' .grad -- so any torch
    optimiser (LBFGS, Adam) steps identically on every rank.  Summation order
    differs from a single-process run: equal within fp32 tolerance.

    loss_grad_fn(X, W, b, y) -> (mean loss, dW, db); default the HIP kernel."""

    def __init__(self, model, group=None, loss_grad_fn: Optional[Callable] = None):
        self.model = model
        self.group = group
        if loss_grad_fn is None:
            from .propagate import linear_xent
            loss_grad_fn = linear_xent
        self.loss_grad_fn = loss_grad_fn

    def loss(self, X_local, y_local, m_global):
        W, b = self.model.W.weight, self.model.W.bias
        C, F = W.shape
        m = int(X_local.shape[0])
        if m > 0:
            loss, dW, db = self.loss_grad_fn(X_local, W.detach(), None if b is None else b.detach(),
                                             y_local)
        else:
            loss, dW = W.new_zeros(()), torch.zeros_like(W)
            db = None if b is None else torch.zeros_like(b)
        scale = m / float(m_global)
        parts = [loss.reshape(1), dW.reshape(-1)] + ([db.reshape(-1)] if b is not None else [])
        buf = torch.cat([t.to(W.dtype) for t in parts]) * scale
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group)
        W.grad = buf[1:1 + C * F].view(C, F).clone()
        if b is not None:
            b.grad = buf[1 + C * F:].clone()
        return buf[0].clone()
