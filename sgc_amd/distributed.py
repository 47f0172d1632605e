"""K-hop propagation across GPUs (one process per GPU): two partitions, two
output layouts, and the data-parallel classifier that consumes them.

RowPartitionedPropagator (the north star's layout, the
default of bench.py --gpus N): each output row of S.X is an independent FMA chain, so the
hot path shards by 1-D row slicing of S.  Rank p owns rows [r_p, r_{p+1}),
chosen by equal nonzero count (prefix of row_ptr) so power-law hubs do not
unbalance the ranks, and computes those rows of X_{k+1} with the same HIP
kernel (sgc_spmm_csr_f32 over a row range, global column indices).  Between
hops every rank needs all of X_k (at Reddit/RMAT shape nearly every column is
referenced by every row block), so the exchange is one all-gather of the row
blocks per hop -- RCCL over xGMI with the "nccl" backend (gloo in the CPU
tests).  Blocks are equal row ranges of B = ceil(N/P) rows (the last one
shorter), so all_gather_into_tensor lands row j of X_k at row j of the
gathered [P*B, Fg] buffer: the next hop reads it with the original column
indices, and no padding crosses xGMI except the last block's tail.  (Equal
rows rather than equal nonzeros: the exchange, not the SpMM, bounds the hop at
large P, and on the randomly labelled Reddit-shape graph equal rows leave the
nonzeros within 5% of balanced at P=8; nnz_balanced_bounds is kept for
graphs where they are not.)

Overlap: features are processed in groups (independent FMA chains, so any
grouping is bit-exact).  Each group's local SpMM is followed by that group's
asynchronous all-gather, so RCCL moves group g while the SpMM computes group
g+1, and the next hop waits only for its own group.

FeaturePartitionedPropagator: S.X acts on each feature column independently,
so rank p owns a block of feature columns and runs all K hops over the full S
with no exchange between hops (see its docstring for the measured trade-off).

Output: "replicated" (every rank gets all of X_K) or "sharded" (every rank
keeps its equal-row block of X_K, which is what ShardedSGCTrainer -- the
data-parallel SGC classifier -- consumes; no full X_K is ever materialised).
"""
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


@dataclass
class ShardCSR:
    """One rank's rows of S (row_ptr rebased to 0, global column indices)."""
    rank: int
    world_size: int
    bounds: np.ndarray      # [P+1] row boundaries
    row_ptr: torch.Tensor   # int32 [rows+1]
    col_idx: torch.Tensor   # int32 [nnz_local]
    val: torch.Tensor       # float32 [nnz_local]
    n: int

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
        return max(1, -(-self.n // self.world_size))


def equal_row_bounds(n, world_size):
    """r_p = min(p * ceil(n/P), n): equal blocks, the last one shorter."""
    B = max(1, -(-n // world_size))
    return np.minimum(np.arange(world_size + 1, dtype=np.int64) * B, n)


def make_shard(row_ptr, col_idx, val, rank, world_size, device):
    """Slice the host CSR (numpy) for `rank` and move it to `device`."""
    row_ptr = np.asarray(row_ptr, dtype=np.int64)
    n = row_ptr.shape[0] - 1
    bounds = equal_row_bounds(n, world_size)
    r0, r1 = int(bounds[rank]), int(bounds[rank + 1])
    k0, k1 = int(row_ptr[r0]), int(row_ptr[r1])

    def t(a, dt):
        return torch.from_numpy(np.ascontiguousarray(a)).to(device=device, dtype=dt)

    return ShardCSR(rank, world_size, bounds, t(row_ptr[r0:r1 + 1] - k0, torch.int32),
                    t(np.asarray(col_idx[k0:k1]), torch.int32),
                    t(np.asarray(val[k0:k1]), torch.float32), n)


def _default_spmm(shard: ShardCSR, X, out):
    from .propagate import DeviceCSR, spmm
    cache = shard.__dict__.setdefault("_csr_by_cols", {})  # hop 1 reads N rows, later P*B
    csr = cache.get(X.shape[0])
    if csr is None:
        csr = DeviceCSR(shard.rows, X.shape[0], shard.row_ptr, shard.col_idx, shard.val)
        cache[X.shape[0]] = csr
    return spmm(csr, X, 0, shard.rows, out=out)


class RowPartitionedPropagator:
    """X_K = S^K X_0 with S row-sharded over the process group.

    X_0 must be the full [N, F] features on every rank (inputs replicated, as
    the reference loads them); the result is the full X_K on every rank.
    `spmm_fn(shard, X, out)` computes the rank's rows of S.X; the default is the
    HIP kernel (tests inject the CPU oracle to exercise the exchange logic over
    gloo).  On the GPU the feature width is padded to a multiple of 32 floats
    inside the engine (128-B rows in every exchanged buffer; the padding
    columns are computed and never returned)."""

    def __init__(self, shard: ShardCSR, group=None, spmm_fn: Optional[Callable] = None,
                 group_floats: int = 224, host_staging: bool = False,
                 pad_input: Optional[bool] = None):
        self.shard = shard
        # Re-lay X_0 into 128-B rows before hop 1?  The copy (all N rows, ~0.2 ms
        # at Reddit shape) beats reading 8-B aligned rows only while this rank's
        # hop-1 share is large: unaligned reads cost +10-18% of that hop
        # (profiles/r01_unaligned_input_sweep.log), so None = pad up to P = 4.
        self.pad_input = pad_input
        self.group = group
        self.spmm_fn = spmm_fn or _default_spmm
        self.group_floats = max(2, int(group_floats) // 2 * 2)  # 8-B aligned groups
        # rehearsal only: gather device buffers through host copies (gloo)
        self.host_staging = host_staging
        self._bufs = {}

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

    def autotune(self, X0, K, output="sharded", candidates=(224, 304, 160), reps=2):
        """Pick group_floats by timing whole propagations (collective: every
        rank must call it with the same arguments).  The best grouping depends
        on the exchange rate, which only the node knows: with a fast all-gather
        the hop after it is compute-bound and fewer, wider groups (cheaper
        launches) win; with a slow one more groups hide more of it
        (DESIGN.md 6).  Each candidate's time is the max over ranks, so every
        rank picks the same width (the all-gathers' shapes must agree).
        Returns {group_floats: seconds per propagation}."""
        import time

        def sync():
            if X0.is_cuda:
                torch.cuda.synchronize(X0.device)
            dist.barrier(group=self.group)

        on_dev = X0.is_cuda and dist.get_backend(self.group) == "nccl"
        times = {}
        for gf in candidates:
            self.group_floats = max(2, int(gf) // 2 * 2)
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
            times[self.group_floats] = float(t.item())
        self.group_floats = min(times, key=lambda g: (times[g], g))
        self._bufs.clear()
        return times

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
        groups = [(a, min(Fp, a + self.group_floats)) for a in range(0, Fp, self.group_floats)]
        src = [X0[:, a:min(b, X0.shape[1])] for a, b in groups]  # unpadded: last one narrower
        works = [None] * len(groups)
        if output == "sharded":
            K_ex = K - 1  # hops whose output is exchanged
            if out is None:
                out = torch.empty((s.rows, F), dtype=torch.float32, device=X0.device)
        else:
            K_ex = K
        for h in range(K_ex):
            par = h & 1
            new_works, gathered = [], []
            for gi, (a, b) in enumerate(groups):
                if works[gi] is not None:
                    works[gi].wait()  # this hop's input group has arrived (stream wait)
                loc = self._buf(("local", par, gi), (s.block, b - a), X0)
                if s.rows:
                    self.spmm_fn(s, src[gi], loc[:s.rows, :src[gi].shape[1]])
                full = self._buf(("full", par, gi), (s.world_size * s.block, b - a), X0)
                new_works.append(self._all_gather(full, loc))
                gathered.append(full)
            works, src = new_works, gathered
        if output == "sharded":
            # last hop: each group straight into this rank's rows of X_K
            for gi, (a, b) in enumerate(groups):
                if works[gi] is not None:
                    works[gi].wait()
                bb = min(b, F)
                if bb > a and s.rows:
                    self.spmm_fn(s, src[gi][:, :bb - a], out[:, a:bb])
            return out
        for w in works:
            if w is not None:
                w.wait()
        if out is None:
            out = torch.empty((n, F), dtype=torch.float32, device=X0.device)
        for gi, (a, b) in enumerate(groups):
            bb = min(b, F)
            if bb > a:
                out[:, a:bb].copy_(src[gi][:n, :bb - a])
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

    spmm_fn(X, row_begin, row_end, out) computes rows [row_begin, row_end) of
    S.X for the columns X has; the default is the HIP kernel over the cached
    DeviceCSR (tests inject the CPU oracle to run the exchange over gloo)."""

    def __init__(self, csr=None, rank=None, world_size=None, group=None,
                 spmm_fn: Optional[Callable] = None, chunks: int = 4,
                 host_staging: bool = False, align: int = 4):
        self.group = group
        self.rank = dist.get_rank(group) if rank is None else int(rank)
        self.world_size = dist.get_world_size(group) if world_size is None else int(world_size)
        if spmm_fn is None:
            if csr is None:
                raise ValueError("FeaturePartitionedPropagator needs a DeviceCSR or an spmm_fn")
            from .propagate import spmm

            def spmm_fn(X, r0, r1, out, _csr=csr):
                return spmm(_csr, X, r0, r1, out=out)
        self.csr = csr
        self.spmm_fn = spmm_fn
        self.chunks = max(1, int(chunks))
        self.align = max(1, int(align))
        self.host_staging = host_staging  # rehearsal only: gathers through host copies (gloo)
        self._bufs = {}

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
        # hops 1..K-1 on the rank's column block, ping-pong in compact buffers
        if K > 1:
            a = self._buf("a", (n, ld), X0)
            _copy_cols(X0[:, c0:c1], a[:, :w])
            src = a[:, :w]
            for h in range(K - 1):
                dst = self._buf(("h", h & 1), (n, ld), X0)[:, :w]
                if w and n:
                    self.spmm_fn(src, 0, n, dst)
                src = dst
        else:
            src = X0[:, c0:c1]  # K = 1: read the block in place
        if output == "sharded":
            # last hop per destination row block -> one all-to-all
            Bn = max(1, -(-n // P))
            send = self._buf("send", (P * Bn, B), X0)
            for q in range(P):
                r0, r1 = int(rb[q]), int(rb[q + 1])
                if w and r1 > r0:
                    self.spmm_fn(src, r0, r1, send[q * Bn:q * Bn + (r1 - r0), :w])
            recv = self._buf("recv", (P * Bn, B), X0)
            work = self._all_to_all(recv, send)
            if work is not None:
                work.wait()
            rows = int(rb[p + 1] - rb[p])
            for q in range(P):
                q0, q1 = int(bounds[q]), int(bounds[q + 1])
                if q1 > q0 and rows:
                    _copy_cols(recv[q * Bn:q * Bn + rows, :q1 - q0], out[:, q0:q1])
            return out
        # last hop in row chunks, each gathered as soon as it is computed
        pending = []
        for ci, (r0, r1) in enumerate(row_chunks(n, self.chunks)):
            rows = r1 - r0
            loc = self._buf(("loc", ci), (rows, B), X0)
            if w and rows:
                self.spmm_fn(src, r0, r1, loc[:, :w])
            full = self._buf(("full", ci), (P * rows, B), X0)
            pending.append((r0, r1, full, self._all_gather(full, loc) if rows else None))
        for r0, r1, full, work in pending:
            if work is not None:
                work.wait()  # the compute stream waits for this chunk's gather
            rows = r1 - r0
            for q in range(P):
                q0, q1 = int(bounds[q]), int(bounds[q + 1])
                if q1 > q0 and rows:
                    _copy_cols(full[q * rows:(q + 1) * rows, :q1 - q0], out[r0:r1, q0:q1])
        return out


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
