"""Row-partitioned K-hop propagation across GPUs (one process per GPU).

SURVEY.md 8(e): each output row of S.X is an independent FMA chain, so the
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
                 group_floats: int = 128, host_staging: bool = False):
        self.shard = shard
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

    def propagate(self, X0, K, out=None):
        s = self.shard
        n, F = X0.shape
        if K <= 0:
            return X0
        Fp = F
        if X0.is_cuda:
            from . import _lib
            from .propagate import aligned_ld
            Fp = aligned_ld(F)
            Xa = self._buf("x0", (n, Fp), X0)  # 128-B rows (propagate() does the same)
            _lib.check(_lib.load().sgc_pad_rows_f32(
                _lib.ptr(X0), X0.stride(0), _lib.ptr(Xa), Fp, n, F,
                _lib.stream_handle(X0.device)), "pad_rows_f32")
            X0 = Xa
        groups = [(a, min(Fp, a + self.group_floats)) for a in range(0, Fp, self.group_floats)]
        src = [X0[:, a:b] for a, b in groups]
        works = [None] * len(groups)
        for h in range(K):
            par = h & 1
            new_works, gathered = [], []
            for gi, (a, b) in enumerate(groups):
                if works[gi] is not None:
                    works[gi].wait()  # this hop's input group has arrived (stream wait)
                loc = self._buf(("local", par, gi), (s.block, b - a), X0)
                if s.rows:
                    self.spmm_fn(s, src[gi], loc[:s.rows])
                full = self._buf(("full", par, gi), (s.world_size * s.block, b - a), X0)
                new_works.append(self._all_gather(full, loc))
                gathered.append(full)
            works, src = new_works, gathered
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
