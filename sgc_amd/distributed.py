"""Row-partitioned K-hop propagation across GPUs (one process per GPU).

SURVEY.md 8(e): each output row of S.X is an independent FMA chain, so the
hot path shards by 1-D row slicing of S.  Rank p owns rows [r_p, r_{p+1}),
chosen by equal nonzero count (prefix of row_ptr) so power-law hubs do not
unbalance the ranks, and computes those rows of X_{k+1} with the same HIP
kernel (sgc_spmm_csr_f32 over a row range).  Between hops every rank needs
all of X_k (at Reddit/RMAT shape nearly every column is referenced by every
row block), so the exchange is one all-gather of the row blocks per hop --
RCCL over xGMI with the "nccl" backend; gloo in the CPU tests.  The exchange
is pipelined against the SpMM by feature groups (RowPartitionedPropagator).

Layout trick: blocks are padded to the largest block (all_gather_into_tensor
needs equal sizes) and the local CSR's column indices are remapped ONCE to
the padded row index  pad(j) = p(j)*block + (j - r_{p(j)}).  The gathered
buffer is then X_{k+1} as the next hop reads it -- no per-hop compaction.
pad() is strictly increasing in j, so every row keeps its column order and
the result stays bit-identical to the single-GPU (and reference) result.
Hop 1 reads the caller's unpadded X_0 with the original indices; the final
hop's blocks are compacted into the [N, F] output.
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
    """One rank's rows of S, with global and padded column indices."""
    rank: int
    world_size: int
    bounds: np.ndarray      # [P+1] row boundaries
    block: int              # padded rows per rank
    row_ptr: torch.Tensor   # int32 [rows+1], rebased to 0
    col_global: torch.Tensor  # int32 [nnz_local]
    col_padded: torch.Tensor  # int32 [nnz_local]
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


def make_shard(row_ptr, col_idx, val, rank, world_size, device):
    """Slice the host CSR (numpy) for `rank` and move it to `device`."""
    row_ptr = np.asarray(row_ptr, dtype=np.int64)
    n = row_ptr.shape[0] - 1
    bounds = nnz_balanced_bounds(row_ptr, world_size)
    sizes = np.diff(bounds)
    block = int(max(1, sizes.max()))
    r0, r1 = int(bounds[rank]), int(bounds[rank + 1])
    k0, k1 = int(row_ptr[r0]), int(row_ptr[r1])
    cols = np.asarray(col_idx[k0:k1], dtype=np.int64)
    owner = np.searchsorted(bounds, cols, side="right") - 1
    padded = owner * block + (cols - bounds[owner])
    if padded.size and padded.max() >= 2**31:
        raise ValueError("padded index exceeds int32")

    def t(a, dt):
        return torch.from_numpy(np.ascontiguousarray(a)).to(device=device, dtype=dt)

    return ShardCSR(rank, world_size, bounds, block, t(row_ptr[r0:r1 + 1] - k0, torch.int32),
                    t(cols, torch.int32), t(padded, torch.int32),
                    t(np.asarray(val[k0:k1]), torch.float32), n)


def _default_spmm(shard: ShardCSR, col, X, out):
    from .propagate import DeviceCSR, spmm
    key = "_csr_padded" if col is shard.col_padded else "_csr_global"
    csr = getattr(shard, key, None)
    if csr is None:
        csr = DeviceCSR(shard.rows, X.shape[0], shard.row_ptr, col, shard.val)
        setattr(shard, key, csr)
    return spmm(csr, X, 0, shard.rows, out=out)


class RowPartitionedPropagator:
    """X_K = S^K X_0 with S row-sharded over the process group.

    X_0 must be the full [N, F] features on every rank (inputs replicated, as
    the reference loads them); the result is the full X_K on every rank.

    Communication/compute overlap: features are processed in groups of
    `group_floats` columns (independent FMA chains, so any grouping is
    bit-exact).  For each hop, group g's local SpMM is followed by an
    asynchronous all-gather of that group (RCCL runs on its own stream), so
    the exchange of group g overlaps the SpMM of group g+1, and the next hop's
    group g only waits for its own gather.  `spmm_fn(shard, col_idx, X, out)`
    computes the rank's rows; the default is the HIP kernel (tests inject the
    CPU oracle to exercise the exchange logic over gloo)."""

    def __init__(self, shard: ShardCSR, group=None, spmm_fn: Optional[Callable] = None,
                 group_floats: int = 128, host_staging: bool = False):
        self.shard = shard
        self.group = group
        self.spmm_fn = spmm_fn or _default_spmm
        self.group_floats = max(2, int(group_floats) // 2 * 2)  # keep 8-B aligned groups
        # rehearsal only: gather device buffers through host copies (gloo)
        self.host_staging = host_staging
        self._bufs = {}

    def _all_gather(self, dst, loc):
        if not self.host_staging:
            return dist.all_gather_into_tensor(dst, loc, group=self.group, async_op=True)
        h_dst = torch.empty(dst.shape, dtype=dst.dtype)
        dist.all_gather_into_tensor(h_dst, loc.cpu(), group=self.group)
        dst.copy_(h_dst)
        return None

    def _buf(self, key, shape, like):
        b = self._bufs.get(key)
        if b is None or tuple(b.shape) != tuple(shape) or b.device != like.device:
            b = torch.empty(shape, dtype=torch.float32, device=like.device)
            self._bufs[key] = b
        return b

    def local_hop(self, X, padded_input, out):
        col = self.shard.col_padded if padded_input else self.shard.col_global
        return self.spmm_fn(self.shard, col, X, out)

    def propagate(self, X0, K, out=None):
        s = self.shard
        P, B = s.world_size, s.block
        F = X0.shape[1]
        if K <= 0:
            return X0
        groups = [(a, min(F, a + self.group_floats)) for a in range(0, F, self.group_floats)]
        if X0.is_cuda:
            from .propagate import aligned_ld, _needs_pad
            if _needs_pad(X0):  # 128-B aligned rows for hop 1's gathers (as propagate())
                from . import _lib
                Xa = self._buf("x0_aligned", (X0.shape[0], aligned_ld(F)), X0)
                _lib.check(_lib.load().sgc_pad_rows_f32(
                    _lib.ptr(X0), X0.stride(0), _lib.ptr(Xa), Xa.stride(0), X0.shape[0], F,
                    _lib.stream_handle(X0.device)), "pad_rows_f32")
                X0 = Xa[:, :F]
        src = [X0[:, a:b] for a, b in groups]
        padded = False
        works = [None] * len(groups)
        for h in range(K):
            par = h & 1
            new_works, gathered = [], []
            for gi, (a, b) in enumerate(groups):
                if works[gi] is not None:
                    works[gi].wait()  # this hop's input group has arrived (stream wait)
                loc = self._buf(("local", par, gi), (B, b - a), X0)
                self.local_hop(src[gi], padded, loc[:s.rows])
                dst = self._buf(("gathered", par, gi), (P * B, b - a), X0)
                new_works.append(self._all_gather(dst, loc))
                gathered.append(dst)
            works, src, padded = new_works, gathered, True
        for w in works:
            if w is not None:
                w.wait()
        if out is None:
            out = torch.empty((s.n, F), dtype=torch.float32, device=X0.device)
        for p in range(P):
            r0, r1 = int(s.bounds[p]), int(s.bounds[p + 1])
            if r1 > r0:
                for gi, (a, b) in enumerate(groups):
                    out[r0:r1, a:b].copy_(src[gi][p * B:p * B + (r1 - r0)])
        return out
