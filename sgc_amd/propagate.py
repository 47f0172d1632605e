"""Device CSR, SpMM and K-hop propagation on gfx950 through libsgc_amd.so.

This is the engine under the drop-in `sgc_precompute` (reference
utils.py:92-97).  Host code only marshals torch tensors into the C ABI
(include/sgc_amd.h); every byte of arithmetic runs in the HIP kernels for
ROCm tensors, and in the library's host twins (sgc_*_cpu, C++ threads) for
CPU tensors -- the reference's own CPU mode (args.py:39 --no-cuda).  A ROCm
tensor never takes the CPU path: mixed devices raise, as torch.spmm does.
"""
import os
from dataclasses import dataclass, field
from typing import NamedTuple, Optional

import numpy as np
import torch

from . import _lib

# Schedule (results never depend on it; see sgc_plan_build): rows with more
# nonzeros than the heavy threshold are split into per-feature-chunk work
# items and scheduled first; rows above the hub threshold run on the LDS-
# staged hub kernel.  Both default to the launch's size, because what they
# bound is the tail -- one wave walking a long row with ~16 nonzeros in flight
# -- against the launch's duration (nnz x F bytes):
#   heavy = nnz*F / 2^23 to the nearest power of two, clamped to [64, 512];
#   hub   = max(heavy, nnz / 1024, 256), capped at 8,192 below 16 M nonzeros.
# The cap (round 2): half of Reddit (11.7 M nonzeros, a P = 2 rank) with
# nnz / 1024 = 11.4k leaves its ~11.5k-nonzero rows as one-wave heavy items
# whose latency outlasts the rank's slice passes -- 2.66 ms per hop vs 2.43
# with hubs above 8,192 (96 rows); the whole graph (19 vs 172 hubs) and a
# quarter (52 either way) are unchanged (profiles/r02/p24_hub_sweep.log).
# Measured (scripts/sweep_narrow.py, profiles/r01_heavy_threshold_sweep.log,
# r01_rank_work_threshold_sweep.log): Reddit full graph 512 / ~10 hubs (988
# hubs cost +20%); a 1/8 row block 128-256 / its 132 rows above 2,048
# (-25% vs. no hubs); Pubmed shape 64 / 16 hubs (-25% vs. 512); Cora shape
# 64 / no hubs (-50%: a 1024-thread hub block costs more than a ~170-nonzero
# row on one wave).  SGC_AMD_HEAVY_THRESHOLD / SGC_AMD_HUB_THRESHOLD pin them.
_HEAVY_ENV = os.environ.get("SGC_AMD_HEAVY_THRESHOLD")
DEFAULT_HEAVY_THRESHOLD = int(_HEAVY_ENV) if _HEAVY_ENV else None
_HUB_ENV = os.environ.get("SGC_AMD_HUB_THRESHOLD")
DEFAULT_HUB_THRESHOLD = int(_HUB_ENV) if _HUB_ENV else None
HUB_SHARE = 1024
HUB_CAP, HUB_CAP_BELOW_NNZ = 8192, 1 << 24


def auto_heavy_threshold(nnz_range, width):
    import math
    work = max(1.0, int(nnz_range) * max(1, int(width)) / float(1 << 23))
    return int(min(512, max(64, 1 << int(round(math.log2(work))))))


def auto_hub_threshold(nnz_range, heavy_threshold):
    hub = int(nnz_range) // HUB_SHARE
    if int(nnz_range) < HUB_CAP_BELOW_NNZ:
        hub = min(hub, HUB_CAP)
    return max(int(heavy_threshold), hub, 256)


class Plan(NamedTuple):
    rows: Optional[torch.Tensor]  # int32 heavy rows, heaviest first (None: no plan)
    n_heavy: int
    n_hub: int
    threshold: int
    max_hub_degree: int = 0  # nonzeros of the longest hub row (0: no hub rows)
    ordered: bool = False  # rows also lists the light rows, longest first (SPMM_LIGHT_ORDER)

    def hub_flags(self):
        """The plan's launch flags: SPMM_HUB_SERIAL when the hub kernel is
        short enough to run in line, SPMM_LIGHT_ORDER when `rows` carries the
        light rows' order."""
        f = SPMM_HUB_SERIAL if 0 < self.max_hub_degree <= HUB_SERIAL_MAX_DEGREE else 0
        return f | (SPMM_LIGHT_ORDER if self.ordered else 0)


NO_PLAN = Plan(None, 0, 0, 0)

SLOT_FIXED, SLOT_X0, SLOT_OUT = 0, 1, 2  # sgc_launch_list_* pointer slots
SPMM_X_PADDED = 1  # sgc_spmm_csr_f32_ex flags (include/sgc_amd.h)
SPMM_Y_PADDED = 2
SPMM_NO_HUB = 4    # split launch: every row but the plan's hub rows
SPMM_HUB_ONLY = 8  # split launch: only the hub rows, on the current stream
SPMM_ACCUMULATE = 16  # column-block pass: continue the chains stored in out
SPMM_HUB_SERIAL = 32  # hub kernel before the light kernel on the same stream
SPMM_LIGHT_ORDER = 64  # plan rows = heavy rows + the light rows in processing order
SPMM_X_UNDER_4G = 128  # X spans < 4 GiB: the gathers may use 32-bit row offsets


def x_flags(X):
    """SPMM_X_UNDER_4G when X has < 2^24 rows and every row lies within 4 GiB
    of its first element (X.shape[0] is the CSR's column count, checked by
    the callers)."""
    n, ld = X.shape[0], X.stride(0)
    return SPMM_X_UNDER_4G if n < (1 << 24) and n * ld * 4 < (1 << 32) else 0
# Light rows of the multi-row kernel in length order (longest first), so the
# rows sharing a wavefront have about the same length: a wave runs to its
# longest row and the other rows' lanes re-load their last nonzero meanwhile
# (the texture-address unit is ~86% busy on the Reddit hop, so those loads
# cost time, profiles/r02/diag).  SGC_AMD_LIGHT_ORDER=0 keeps row order.
LIGHT_ORDER = os.environ.get("SGC_AMD_LIGHT_ORDER", "1") != "0"
# Longest hub row (nonzeros) for which the serial hub launch beats the
# side-stream fork/join: its chain (~6.4 ns per nonzero) plus a
# launch stays under the ~25 us the two cross-stream events cost.
HUB_SERIAL_MAX_DEGREE = 3072

STATUS_ROWS_SORTED = 1
STATUS_COLS_ASCENDING = 2
STATUS_OUT_OF_RANGE = 4

# Column groups (sgc_csr_colsplit): one hop as G launches over the same rows,
# group 0 plain and groups 1.. accumulating, each gathering only the X rows
# of its column range -- the live X slice is 1/G as large and more of it stays
# in the per-XCD L2s.  Same bits (rows with ascending columns only).  Measured
# one hop, interleaved, bit-identical (profiles/r03/s14/colgroup*.log):
# Reddit shape at 602 floats 4.30 -> 3.83 ms (G = 2; 3.81 at 3, 3.88 at 4, 4.73
# at 8), at 304 2.45 -> 2.29, at 128 0.95 -> 0.84, at 76 0.77 -> 0.77, at
# 152 / 256 (the one-row kernel) 1.56 -> 1.58 / 1.85 -> 1.88;
# RMAT shape (F = 256) 31.4 -> 30.1 (G = 2) -> 29.5 ms (G = 4).  None set =
# column_groups_for's size rule; SGC_AMD_COLUMN_GROUPS=G forces G (1 = off).
_GROUPS_ENV = os.environ.get("SGC_AMD_COLUMN_GROUPS")
COLUMN_GROUPS = int(_GROUPS_ENV) if _GROUPS_ENV else None
GROUPS_MIN_NNZ = 1 << 22    # below: latency-bound launches, one launch per hop
GROUPS_MIN_WIDTH = 128      # narrower launches gain nothing (76 floats: 0.77 vs 0.77 ms)
GROUPS_WIDE_NNZ = 1 << 26   # from here four groups (RMAT shape)


def column_groups_for(csr, width):
    """Column groups for a plain launch of `width` features over `csr`."""
    if csr.device.type != "cuda" or not csr.cols_ascending or csr.nnz == 0:
        return 1
    if COLUMN_GROUPS is not None:
        return max(1, min(8, int(COLUMN_GROUPS), max(1, csr.n_cols)))
    if width < GROUPS_MIN_WIDTH or csr.nnz < GROUPS_MIN_NNZ:
        return 1
    if csr.nnz >= GROUPS_WIDE_NNZ:
        return 4
    if 128 < width <= 256:  # the one-row kernel's single 256-float slice: no gain
        return 1            # (152 floats 1.56 -> 1.58 ms, 256 1.85 -> 1.88 at G = 2)
    return 2


def _host_cols_ascending(row_ptr, col_idx):
    """Every row's columns strictly ascending?  (host arrays; False for
    anything else, which only turns the column groups off)."""
    if isinstance(row_ptr, torch.Tensor):
        if row_ptr.device.type != "cpu" or col_idx.device.type != "cpu":
            return False
        row_ptr, col_idx = row_ptr.numpy(), col_idx.numpy()
    rp = np.asarray(row_ptr, dtype=np.int64)
    ci = np.asarray(col_idx)
    if ci.size < 2:
        return True
    bad = np.diff(ci.astype(np.int64)) <= 0  # bad[k-1]: col[k] <= col[k-1]
    starts = rp[1:-1]
    starts = starts[(starts > 0) & (starts < ci.size)]
    bad[starts - 1] = False  # k is a row's first nonzero: no predecessor in its row
    return not bool(bad.any())


def _require_device(t, what):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"sgc_amd: {what} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise RuntimeError(
            f"sgc_amd: {what} is on {t.device}; the propagation engine runs only on a "
            "ROCm (gfx950) device -- move tensors with .cuda() (no CPU fallback)")


def cpu_threads():
    """Threads of the host path: torch's intra-op setting (torch.set_num_threads)."""
    return max(1, torch.get_num_threads())


@dataclass
class DeviceCSR:
    """int32 CSR of the normalised adjacency S, resident in HBM (or in host
    memory for a CPU adjacency).

    Built once per adjacency tensor (cached on it) by a stable sort of the
    COO entries by row: every stored entry is kept and each row keeps its
    storage order, which is the FMA order of torch.spmm's CPU kernel."""
    n_rows: int
    n_cols: int
    row_ptr: torch.Tensor  # int32 [n_rows+1]
    col_idx: torch.Tensor  # int32 [nnz]
    val: torch.Tensor      # float32 [nnz]
    status: int = 0
    ingest_seconds: float = 0.0
    _plans: dict = field(default_factory=dict)

    @property
    def nnz(self):
        return self.col_idx.numel()

    @property
    def device(self):
        return self.row_ptr.device

    @property
    def cols_ascending(self):
        """Every row's columns strictly ascending (the ingest's status bit)."""
        return bool(self.status & STATUS_COLS_ASCENDING)

    def group_cuts(self, G):
        """Column cuts of the G column groups: group g = columns [c_g, c_{g+1})."""
        return [(g * self.n_cols) // G for g in range(G + 1)]

    def column_groups(self, G):
        """The G column-group CSRs of this one (sgc_csr_colsplit; cached):
        columns cut at g * n_cols / G, every row's run of each group in its
        storage order; group g's row_ptr points into one shared col/val
        copy.  Rows must have ascending columns."""
        if not self.cols_ascending:
            raise ValueError("sgc_amd: column groups need rows with ascending columns")
        key = ("groups", int(G))
        if key not in self._plans:
            import ctypes
            lib = _lib.load()
            n, nnz, dev = self.n_rows, self.nnz, self.device
            cuts = (ctypes.c_int32 * (G + 1))(*self.group_cuts(G))
            row_ptrs = torch.empty((G, n + 1), dtype=torch.int32, device=dev)
            col = torch.empty(max(1, nnz), dtype=torch.int32, device=dev)
            val = torch.empty(max(1, nnz), dtype=torch.float32, device=dev)
            ws_bytes = lib.sgc_colsplit_workspace(n, G)
            ws = torch.empty(max(1, ws_bytes), dtype=torch.uint8, device=dev)
            with torch.cuda.device(dev):
                _lib.check(lib.sgc_csr_colsplit(_lib.ptr(self.row_ptr), _lib.ptr(self.col_idx),
                                                _lib.ptr(self.val), n, self.n_cols, G,
                                                ctypes.cast(cuts, ctypes.c_void_p),
                                                _lib.ptr(row_ptrs), _lib.ptr(col), _lib.ptr(val),
                                                _lib.ptr(ws), ws_bytes,
                                                _lib.stream_handle(dev)), "csr_colsplit")
            del ws  # stream-ordered: the allocator reuses it after the kernels
            self._plans[key] = [DeviceCSR(n, self.n_cols, row_ptrs[g], col[:nnz], val[:nnz],
                                          self.status) for g in range(G)]
        return self._plans[key]

    def release_prepared(self):
        """Free propagate()'s recorded launch lists on this adjacency (each
        keeps its launches' arguments and up to PREPARED_LOOP_MAX_BYTES of
        intermediates; at most PREPARED_LOOPS_KEPT of them).  The next call
        records again."""
        for key in [k for k in self._plans if isinstance(k, tuple) and k[:1] == ("list",)]:
            del self._plans[key]

    def drop_groups(self):
        """Free the cached column-group copies of S (and their plans): one
        more col/val copy per G (188 MB at Reddit shape).  They are rebuilt
        on the next launch that uses them."""
        self.release_prepared()  # recorded launch lists hold the groups' pointers
        for key in [k for k in self._plans if isinstance(k, tuple) and k[:1] == ("groups",)]:
            for part in self._plans.pop(key):
                part._plans.clear()

    def groups_or_self(self, G):
        """The G column-group CSRs, or [self] when G == 1 or when the copy
        does not fit in device memory (a schedule: the results are the same)."""
        if G <= 1:
            return [self]
        try:
            return self.column_groups(G)
        except torch.cuda.OutOfMemoryError:
            return [self]

    @classmethod
    def from_host_arrays(cls, row_ptr, col_idx, val, n_cols=None, device="cuda"):
        """From host CSR arrays already in the SpMM's order (numpy or torch)."""
        status = STATUS_COLS_ASCENDING if _host_cols_ascending(row_ptr, col_idx) else 0
        rp = torch.as_tensor(row_ptr).to(device=device, dtype=torch.int32)
        ci = torch.as_tensor(col_idx).to(device=device, dtype=torch.int32)
        va = torch.as_tensor(val).to(device=device, dtype=torch.float32)
        n = rp.numel() - 1
        return cls(n, n if n_cols is None else n_cols, rp.contiguous(), ci.contiguous(),
                   va.contiguous(), status)

    @classmethod
    def from_torch(cls, adj):
        """From a torch sparse COO (reference utils.py:23-30 layout) or CSR tensor."""
        import time
        if isinstance(adj, torch.Tensor) and adj.device.type == "cpu":
            return cls._from_torch_cpu(adj)
        _require_device(adj, "adj")
        if adj.dtype != torch.float32:
            raise TypeError(f"sgc_amd: adj must be float32, got {adj.dtype}")
        if adj.dim() != 2:
            raise ValueError("sgc_amd: adj must be 2-D")
        lib = _lib.load()
        n_rows, n_cols = adj.shape
        dev = adj.device
        t0 = time.perf_counter()
        with torch.cuda.device(dev):
            stream = _lib.stream_handle(dev)
            status = _lib._u32(0)
            if adj.layout == torch.sparse_coo:
                idx = adj._indices().contiguous()
                vals = adj._values().contiguous()
                nnz = vals.numel()
                rows, cols = idx[0], idx[1]
                row_ptr = torch.empty(n_rows + 1, dtype=torch.int32, device=dev)
                col_idx = torch.empty(nnz, dtype=torch.int32, device=dev)
                val = torch.empty(nnz, dtype=torch.float32, device=dev)
                ws_bytes = _lib._sz(0)
                _lib.check(lib.sgc_coo_to_csr_workspace(n_rows, nnz, ctypes_byref(ws_bytes)),
                           "coo_to_csr_workspace")
                ws = torch.empty(max(1, ws_bytes.value), dtype=torch.uint8, device=dev)
                _lib.check(lib.sgc_coo_to_csr(_lib.ptr(rows), _lib.ptr(cols), _lib.ptr(vals), nnz,
                                              n_rows, n_cols, _lib.ptr(row_ptr), _lib.ptr(col_idx),
                                              _lib.ptr(val), _lib.ptr(ws), ws_bytes.value,
                                              ctypes_byref(status), stream), "coo_to_csr")
                del ws
            elif adj.layout == torch.sparse_csr:
                crow = adj.crow_indices().to(torch.int64).contiguous()
                ccol = adj.col_indices().to(torch.int64).contiguous()
                vals = adj.values().contiguous()
                nnz = vals.numel()
                row_ptr = torch.empty(n_rows + 1, dtype=torch.int32, device=dev)
                col_idx = torch.empty(nnz, dtype=torch.int32, device=dev)
                val = torch.empty(nnz, dtype=torch.float32, device=dev)
                _lib.check(lib.sgc_csr64_to_csr(_lib.ptr(crow), _lib.ptr(ccol), _lib.ptr(vals),
                                                nnz, n_rows, n_cols, _lib.ptr(row_ptr),
                                                _lib.ptr(col_idx), _lib.ptr(val),
                                                ctypes_byref(status), stream), "csr64_to_csr")
            else:
                raise TypeError(f"sgc_amd: unsupported adj layout {adj.layout}")
        csr = cls(n_rows, n_cols, row_ptr, col_idx, val, int(status.value))
        csr.ingest_seconds = time.perf_counter() - t0
        return csr

    @classmethod
    def _from_torch_cpu(cls, adj):
        """Host CSR of a CPU adjacency (sgc_coo_to_csr_cpu: stable by row)."""
        import time
        if adj.dtype != torch.float32:
            raise TypeError(f"sgc_amd: adj must be float32, got {adj.dtype}")
        if adj.dim() != 2:
            raise ValueError("sgc_amd: adj must be 2-D")
        lib = _lib.load()
        n_rows, n_cols = adj.shape
        t0 = time.perf_counter()
        if adj.layout == torch.sparse_coo:
            idx = adj._indices().contiguous()
            vals = adj._values().contiguous()
        elif adj.layout == torch.sparse_csr:
            crow = adj.crow_indices().to(torch.int64)
            rows = torch.repeat_interleave(torch.arange(n_rows, dtype=torch.int64),
                                           crow[1:] - crow[:-1])
            idx = torch.stack([rows, adj.col_indices().to(torch.int64)])
            vals = adj.values().contiguous()
        else:
            raise TypeError(f"sgc_amd: unsupported adj layout {adj.layout}")
        nnz = vals.numel()
        row_ptr = torch.empty(n_rows + 1, dtype=torch.int32)
        col_idx = torch.empty(nnz, dtype=torch.int32)
        val = torch.empty(nnz, dtype=torch.float32)
        status = _lib._u32(0)
        _lib.check(lib.sgc_coo_to_csr_cpu(_lib.ptr(idx[0]), _lib.ptr(idx[1]), _lib.ptr(vals), nnz,
                                          n_rows, n_cols, _lib.ptr(row_ptr), _lib.ptr(col_idx),
                                          _lib.ptr(val), ctypes_byref(status)), "coo_to_csr_cpu")
        csr = cls(n_rows, n_cols, row_ptr, col_idx, val, int(status.value))
        csr.ingest_seconds = time.perf_counter() - t0
        return csr

    def range_nnz(self, row_begin, row_end):
        """Nonzeros of rows [row_begin, row_end) (cached; reads row_ptr once)."""
        key = ("nnz", row_begin, row_end)
        if key not in self._plans:
            nnz = 0
            if row_end > row_begin:
                ends = self.row_ptr[[row_begin, row_end]].tolist()
                nnz = ends[1] - ends[0]
            self._plans[key] = nnz
        return self._plans[key]

    def plan(self, row_begin=0, row_end=None, threshold=None, hub_threshold=None,
             width=None) -> Plan:
        """Heavy-row schedule for rows [row_begin, row_end) at `width` features
        (cached).  Thresholds left None take the size-based defaults above."""
        row_end = self.n_rows if row_end is None else row_end
        if threshold is None:
            threshold = DEFAULT_HEAVY_THRESHOLD
        if threshold is None:
            threshold = auto_heavy_threshold(self.range_nnz(row_begin, row_end),
                                             width if width is not None else 512)
        threshold = int(threshold)
        hub = DEFAULT_HUB_THRESHOLD if hub_threshold is None else int(hub_threshold)
        if hub is None:
            hub = auto_hub_threshold(self.range_nnz(row_begin, row_end), threshold)
        hub = max(hub, threshold)
        key = (row_begin, row_end, threshold, hub)
        if key not in self._plans and LIGHT_ORDER and self.device.type == "cuda":
            self._plans[key] = self._plan_sorted(row_begin, row_end, threshold, hub)
        if key not in self._plans:
            lib = _lib.load()
            n = row_end - row_begin
            cap = lib.sgc_plan_capacity(n)
            buf = torch.empty(max(1, cap), dtype=torch.int32, device=self.device)
            n_heavy, n_hub = _lib._i64(0), _lib._i64(0)
            with torch.cuda.device(self.device):
                _lib.check(lib.sgc_plan_build(_lib.ptr(self.row_ptr), row_begin, row_end, threshold,
                                              hub, _lib.ptr(buf), cap, ctypes_byref(n_heavy),
                                              ctypes_byref(n_hub),
                                              _lib.stream_handle(self.device)), "plan_build")
            h, nh = int(n_heavy.value), int(n_hub.value)
            deg = 0
            if nh > 0:  # heaviest first: row 0 of the plan is the longest hub chain
                r = int(buf[0].item())
                ends = self.row_ptr[[r, r + 1]].tolist()
                deg = ends[1] - ends[0]
            rows, ordered = buf[:max(h, 1)].clone(), False
            if LIGHT_ORDER and self.device.type == "cuda" and n > h:
                # plan rows = [heavy rows | light rows longest first]
                rows = torch.empty(n, dtype=torch.int32, device=self.device)
                rows[:h].copy_(buf[:h])
                n_light = _lib._i64(0)
                with torch.cuda.device(self.device):
                    _lib.check(lib.sgc_plan_light_order(
                        _lib.ptr(self.row_ptr), row_begin, row_end, threshold,
                        _lib.ptr(rows[h:]), ctypes_byref(n_light),
                        _lib.stream_handle(self.device)), "plan_light_order")
                if int(n_light.value) != n - h:
                    raise RuntimeError("sgc_amd: light order does not cover the light rows")
                ordered = True
            self._plans[key] = Plan(rows, h, nh, threshold, deg, ordered)
        return self._plans[key]


    def _plan_sorted(self, row_begin, row_end, threshold, hub):
        """The plan from one device radix sort (sgc_plan_sorted): all rows of
        the range by degree, longest first -- heavy rows, then the light rows
        in processing order -- and the counts in one read-back."""
        import ctypes
        lib = _lib.load()
        n = row_end - row_begin
        rows = torch.empty(max(1, n), dtype=torch.int32, device=self.device)
        ws_bytes = lib.sgc_plan_sorted_workspace(n)
        ws = torch.empty(max(1, ws_bytes), dtype=torch.uint8, device=self.device)
        counts = (ctypes.c_int64 * 3)()
        with torch.cuda.device(self.device):
            _lib.check(lib.sgc_plan_sorted(_lib.ptr(self.row_ptr), row_begin, row_end, threshold,
                                           hub, _lib.ptr(rows), _lib.ptr(ws), ws_bytes,
                                           ctypes.cast(counts, ctypes.c_void_p),
                                           _lib.stream_handle(self.device)), "plan_sorted")
        h, nh = int(counts[0]), int(counts[1])
        return Plan(rows, h, nh, threshold, int(counts[2]) if nh > 0 else 0, n > h)


def to_torch_coo(csr: DeviceCSR):
    """torch sparse COO (int64 [2, nnz] indices, fp32 values, not coalesced) with
    the entries in CSR order -- the tensor sparse_mx_to_torch_sparse_tensor
    (utils.py:23-30) builds -- with `csr` attached as its propagation cache."""
    lib = _lib.load()
    nnz = csr.nnz
    idx = torch.empty((2, nnz), dtype=torch.int64, device=csr.device)
    with torch.cuda.device(csr.device):
        _lib.check(lib.sgc_csr_to_coo64(_lib.ptr(csr.row_ptr), _lib.ptr(csr.col_idx), csr.n_rows,
                                        _lib.ptr(idx[0]), _lib.ptr(idx[1]),
                                        _lib.stream_handle(csr.device)), "csr_to_coo64")
    adj = torch.sparse_coo_tensor(idx, csr.val, (csr.n_rows, csr.n_cols))
    try:
        adj._sgc_amd_csr = (adj._version, csr)
    except (AttributeError, RuntimeError):
        pass
    return adj


def ctypes_byref(x):
    import ctypes
    return ctypes.byref(x)


def csr_of(adj):
    """Cached DeviceCSR of a torch sparse adjacency (rebuilt if adj changed)."""
    cached = getattr(adj, "_sgc_amd_csr", None)
    if cached is not None and cached[0] == adj._version:
        return cached[1]
    csr = DeviceCSR.from_torch(adj)
    try:
        adj._sgc_amd_csr = (adj._version, csr)
    except (AttributeError, RuntimeError):
        pass
    return csr


def _check_features(X, csr):
    if not isinstance(X, torch.Tensor):
        raise TypeError("sgc_amd: features must be a torch.Tensor")
    if csr.device.type != "cpu":
        _require_device(X, "features")
    if X.device != csr.device:
        raise RuntimeError(f"sgc_amd: features on {X.device} but adj on {csr.device}")
    if X.dtype != torch.float32:
        raise TypeError(f"sgc_amd: features must be float32, got {X.dtype}")
    if X.dim() != 2 or X.shape[0] != csr.n_cols:
        raise RuntimeError(f"sgc_amd: size mismatch, adj {csr.n_rows}x{csr.n_cols} . "
                           f"features {tuple(X.shape)}")
    if X.stride(1) != 1 or X.stride(0) < X.shape[1]:
        X = X.contiguous()
    return X


def check_propagation_inputs(csr: DeviceCSR, X: torch.Tensor):
    """The checks propagate() makes (types, devices, shapes, a square S);
    returns X with unit column stride."""
    X = _check_features(X, csr)
    if csr.n_rows != csr.n_cols:
        raise RuntimeError("sgc_amd: propagation needs a square adjacency")
    return X


def spmm(csr: DeviceCSR, X: torch.Tensor, row_begin=0, row_end=None, out=None,
         use_plan=True, threshold=None, hub_threshold=None, flags=0):
    """One hop Y = S[row_begin:row_end] . X (bit-exact with torch.spmm on CPU).
    flags: SPMM_* bits of sgc_spmm_csr_f32_ex (a split launch on the GPU: NO_HUB
    / HUB_ONLY; on the CPU the whole hop runs for the NO_HUB part and nothing
    for HUB_ONLY, so the two parts still write every row once; ACCUMULATE
    continues the FMA chains already in `out`, which must then be given)."""
    X = _check_features(X, csr)
    row_end = csr.n_rows if row_end is None else row_end
    F = X.shape[1]
    if out is None:
        if flags & SPMM_ACCUMULATE:
            raise ValueError("sgc_amd: SPMM_ACCUMULATE continues the chains in `out`; pass it")
        out = torch.empty((row_end - row_begin, F), dtype=torch.float32, device=X.device)
    if F == 0 or row_end == row_begin:
        return out
    lib = _lib.load()
    if X.device.type == "cpu":
        if flags & SPMM_HUB_ONLY:
            return out
        _lib.check(lib.sgc_spmm_csr_f32_cpu_ex(_lib.ptr(csr.row_ptr), _lib.ptr(csr.col_idx),
                                               _lib.ptr(csr.val), row_begin, row_end,
                                               _lib.ptr(X), X.stride(0), _lib.ptr(out),
                                               out.stride(0), F, int(flags) & ~SPMM_NO_HUB,
                                               cpu_threads()), "spmm_csr_f32_cpu")
        return out
    G = 1
    if use_plan and not flags & (SPMM_ACCUMULATE | SPMM_NO_HUB | SPMM_HUB_ONLY):
        G = column_groups_for(csr, F)
    parts = csr.groups_or_self(G)
    with torch.cuda.device(X.device):
        stream = _lib.stream_handle(X.device)
        for g, c in enumerate(parts):  # group 0 plain, groups 1.. continue its chains
            pl = c.plan(row_begin, row_end, threshold, hub_threshold, F) if use_plan else NO_PLAN
            _lib.check(lib.sgc_spmm_csr_f32_ex(_lib.ptr(c.row_ptr), _lib.ptr(c.col_idx),
                                               _lib.ptr(c.val), row_begin, row_end, _lib.ptr(X),
                                               X.stride(0), _lib.ptr(out), out.stride(0), F,
                                               _lib.ptr(pl.rows), pl.n_heavy, pl.n_hub,
                                               pl.threshold,
                                               int(flags) | pl.hub_flags() | x_flags(X) |
                                               (SPMM_ACCUMULATE if g else 0), stream),
                       "spmm_csr_f32")
    return out


class SpmmLaunch:
    """One prepared SpMM launch (fixed CSR, plan, X, out, flags): the ctypes
    arguments are built once and each call only passes the stream.  The
    multi-GPU pipeline replays a dozen launches per step, where the checks
    and lookups of spmm() would cost more host time than the launches take on
    the GPU.  The tensors must stay alive and unchanged in shape/storage;
    keep_tensors=False drops the references to X and out (for caches keyed by
    their data_ptr/shape/stride, which only replay a launch for live tensors
    at those addresses -- so a cache never pins a caller's tensor)."""

    __slots__ = ("_fn", "_args", "_keep")

    def __init__(self, csr: DeviceCSR, X: torch.Tensor, out: torch.Tensor, row_begin=0,
                 row_end=None, flags=0, threshold=None, hub_threshold=None, keep_tensors=True):
        X = _check_features(X, csr)
        if X.device.type != "cuda":
            raise RuntimeError("SpmmLaunch: ROCm tensors only")
        row_end = csr.n_rows if row_end is None else row_end
        F = X.shape[1]
        pl = csr.plan(row_begin, row_end, threshold, hub_threshold, F)
        lib = _lib.load()
        self._fn = lib.sgc_spmm_csr_f32_ex
        self._keep = (csr, X, out, pl) if keep_tensors else (csr, pl)
        self._args = (_lib.ptr(csr.row_ptr), _lib.ptr(csr.col_idx), _lib.ptr(csr.val),
                      int(row_begin), int(row_end), _lib.ptr(X), X.stride(0), _lib.ptr(out),
                      out.stride(0), F, _lib.ptr(pl.rows), pl.n_heavy, pl.n_hub, pl.threshold,
                      int(flags) | pl.hub_flags() | x_flags(X))

    def __call__(self, stream_handle):
        rc = self._fn(*self._args, stream_handle)
        if rc:
            _lib.check(rc, "spmm_csr_f32 (prepared)")


def aligned_ld(F):
    """Row stride (floats) of the engine's own feature buffers: 128-B rows."""
    return (F + 31) // 32 * 32


def _needs_pad(X):
    return X.stride(0) % 32 != 0 or X.data_ptr() % 128 != 0


# Override of pad_pays (None = the rule; True / False force the re-layout on
# or off -- scripts/pad_ab.py times both, results bit-identical either way).
PAD_X0 = None


def pad_pays(csr, F):
    """Re-lay X_0 into 128-B rows before hop 1?  An unaligned row segment
    touches about one extra 128-B line per gathered row (32/F of the hop's
    gather bytes, 128 B per nonzero); the copy moves 8 B per element of X
    (read + write).  With gathers ~1.2x the streaming rate the copy pays when
    16 * nnz/N > 1.2 F: Reddit (degree 100, F 602) and RMAT shape yes,
    Pubmed / Cora shape (degree ~5) no."""
    n = max(1, csr.n_rows)
    return 16.0 * csr.range_nnz(0, csr.n_rows) / n > 1.2 * F


def propagate(csr: DeviceCSR, X: torch.Tensor, K: int, out=None, use_plan=True, threshold=None,
              hop_hook=None, native_loop=False, hub_threshold=None, prepare=True):
    """X_K = S^K X on the device (K >= 1); asynchronous on the current stream.

    Mirrors sgc_propagate_f32: X is first re-laid into 128-B aligned rows when
    its rows are not and the copy pays (pad_pays: one streaming copy; each
    gathered X segment then spans the fewest 128-B lines -- sgc_propagate_f32
    always copies), hops ping-pong between two aligned buffers, the
    last hop writes the contiguous [N, F] result.  hop_hook(phase, h) is called
    around each hop's launch ("start"/"end", for event timing).
    native_loop=True runs the same loop inside the C ABI call instead.
    prepare=False neither replays nor records a launch list (GraphedPropagation's
    warm-up and capture; nothing is kept under a stream capture either)."""
    X = check_propagation_inputs(csr, X)
    n, F = X.shape
    if out is None:
        out = torch.empty((n, F), dtype=torch.float32, device=X.device)
    if n == 0 or F == 0 or K <= 0:
        if K <= 0:
            out.copy_(X)
        return out
    lib = _lib.load()
    if X.device.type == "cpu":  # host twin (reference CPU mode), same bits
        ws_bytes = lib.sgc_propagate_cpu_workspace(n, F, int(K))
        ws = torch.empty(max(1, ws_bytes), dtype=torch.uint8)
        _lib.check(lib.sgc_propagate_f32_cpu(_lib.ptr(csr.row_ptr), _lib.ptr(csr.col_idx),
                                             _lib.ptr(csr.val), n, _lib.ptr(X), X.stride(0),
                                             _lib.ptr(out), out.stride(0), F, int(K), _lib.ptr(ws),
                                             ws_bytes, cpu_threads()), "propagate_f32_cpu")
        return out
    stream = torch.cuda.current_stream(X.device).cuda_stream  # (an int: ctypes takes it as void *)
    G_rule = column_groups_for(csr, F) if use_plan else 1
    # small launches (Cora / Pubmed shape: 20-40 us hops) pay their host time:
    # the loop's launches are recorded once per (shape, strides, X_0's 128-B
    # alignment, K, stream, schedule) into a native launch list, with the
    # intermediates kept beside it, and replayed by one call that takes this
    # call's X_0 and X_K
    key = None
    if (not native_loop and hop_hook is None and prepare and X.data_ptr() != out.data_ptr()
            and not torch.cuda.is_current_stream_capturing()):
        key = ("list", X.stride(0), F, int(K), out.stride(0), X.data_ptr() % 128 == 0,
               threshold, hub_threshold, bool(use_plan), G_rule, stream, PAD_X0)
        prep = csr._plans.get(key)
        if prep is not None:
            rc = lib.sgc_launch_list_run(prep[1].handle, X.data_ptr(), out.data_ptr(), stream)
            if rc:
                _lib.check(rc, "propagate (launch list)")
            return out
    G = len(csr.groups_or_self(G_rule))
    if G > 1:
        pl = None
        parts = [(c, c.plan(0, n, threshold, hub_threshold, F)) for c in csr.column_groups(G)]
    else:
        pl = csr.plan(0, n, threshold, hub_threshold, F) if use_plan else NO_PLAN
        parts = [(csr, pl)]
    # (csr, plan, launch flags of the group): groups 1.. continue group 0's chains
    parts = [(c, cp, cp.hub_flags() | (SPMM_ACCUMULATE if g else 0))
             for g, (c, cp) in enumerate(parts)]
    ldw = aligned_ld(F)
    with torch.cuda.device(X.device):
        if native_loop:  # the same loop inside one C ABI call (sgc_propagate_groups_f32)
            import ctypes
            Gn = len(parts)
            ws_bytes = lib.sgc_propagate_workspace(n, F, X.stride(0), K)
            ws = torch.empty(max(1, ws_bytes), dtype=torch.uint8, device=X.device)
            planned = use_plan and all(cp.rows is not None for _, cp, _ in parts)
            plans = (ctypes.c_void_p * Gn)(*[cp.rows.data_ptr() if planned else None
                                             for _, cp, _ in parts])
            n_heavy = (ctypes.c_int64 * Gn)(*[cp.n_heavy for _, cp, _ in parts])
            n_hub = (ctypes.c_int64 * Gn)(*[cp.n_hub for _, cp, _ in parts])
            ths = (ctypes.c_int32 * Gn)(*[cp.threshold for _, cp, _ in parts])
            pflags = (ctypes.c_uint32 * Gn)(*[cp.hub_flags() for _, cp, _ in parts])
            row_ptrs = parts[0][0].row_ptr  # groups: row 0 of the [G, n+1] row_ptrs tensor
            _lib.check(lib.sgc_propagate_groups_f32(
                Gn, _lib.ptr(row_ptrs), _lib.ptr(parts[0][0].col_idx), _lib.ptr(parts[0][0].val), n,
                _lib.ptr(X), X.stride(0), _lib.ptr(out), out.stride(0), F, int(K),
                ctypes.cast(plans, ctypes.c_void_p) if planned else None,
                ctypes.cast(n_heavy, ctypes.c_void_p), ctypes.cast(n_hub, ctypes.c_void_p),
                ctypes.cast(ths, ctypes.c_void_p), ctypes.cast(pflags, ctypes.c_void_p),
                _lib.ptr(ws), ws_bytes, stream), "propagate_groups_f32")
            return out
        pad = _needs_pad(X) and (pad_pays(csr, F) if PAD_X0 is None else bool(PAD_X0))
        # buffers actually used: the re-laid X_0 (if any) + up to two
        # ping-pong intermediates (the last hop writes `out`)
        n_bufs = min(2, int(pad) + min(K - 1, 2))
        prepared = key is not None and n_bufs * n * ldw * 4 <= PREPARED_LOOP_MAX_BYTES
        bufs = [torch.empty((n, ldw), dtype=torch.float32, device=X.device)
                for _ in range(n_bufs)]
        ops = []  # the launches as recorded: (kind, args without the stream, src slot, dst slot)

        def slot(t):
            return SLOT_X0 if t is X else SLOT_OUT if t is out else SLOT_FIXED
        src, nxt = X, 0
        if pad:
            args = (_lib.ptr(X), X.stride(0), _lib.ptr(bufs[0]), ldw, n, F)
            ops.append(("pad", args, SLOT_X0, SLOT_FIXED))
            src, nxt = bufs[0][:, :F], 1 % len(bufs)
            _lib.check(lib.sgc_pad_rows_f32(*args, stream), "pad_rows_f32")
        for h in range(K):
            dst = out if h == K - 1 else bufs[nxt][:, :F]
            # the engine's own buffers may be read / written in their pad columns
            flags = ((SPMM_X_PADDED if src is not X else 0) |
                     (SPMM_Y_PADDED if dst is not out else 0) | x_flags(src))
            if hop_hook:
                hop_hook("start", h)
            for c, cp, gflags in parts:  # column groups: 0 plain, 1.. accumulate
                args = (_lib.ptr(c.row_ptr), _lib.ptr(c.col_idx), _lib.ptr(c.val), 0, n,
                        _lib.ptr(src), src.stride(0), _lib.ptr(dst), dst.stride(0), F,
                        _lib.ptr(cp.rows), cp.n_heavy, cp.n_hub, cp.threshold, flags | gflags)
                ops.append(("spmm", args, slot(src), slot(dst)))
                _lib.check(lib.sgc_spmm_csr_f32_ex(*args, stream), "spmm_csr_f32")
            if hop_hook:
                hop_hook("end", h)
            src, nxt = dst, nxt ^ 1
        if prepared:
            old = [k for k in csr._plans if isinstance(k, tuple) and k[:1] == ("list",)]
            for k in old[:max(0, len(old) - PREPARED_LOOPS_KEPT + 1)]:
                del csr._plans[k]  # oldest first (dicts keep insertion order)
            csr._plans[key] = (bufs, LaunchList(ops), parts)  # parts: keep the pointers alive
    return out


class LaunchList:
    """A native launch list (sgc_launch_list_*) holding one propagate() loop:
    the ops as recorded, X_0 / X_K by slot; destroyed with this object."""

    __slots__ = ("handle", "_lib")

    def __init__(self, ops):
        import ctypes
        lib = _lib.load()
        h = ctypes.c_int64(0)
        _lib.check(lib.sgc_launch_list_create(ctypes.byref(h)), "launch_list_create")
        self.handle, self._lib = h.value, lib
        for kind, args, s_src, s_dst in ops:
            if kind == "pad":
                rc = lib.sgc_launch_list_add_pad_rows(self.handle, *args, s_src, s_dst)
            else:
                rc = lib.sgc_launch_list_add_spmm(self.handle, *args, s_src, s_dst)
            _lib.check(rc, "launch_list_add")

    def __del__(self):
        try:
            if self.handle:
                self._lib.sgc_launch_list_destroy(self.handle)
                self.handle = 0
        except Exception:  # interpreter shutdown: the library may be gone
            pass


# propagate()'s recorded launch lists: at most this many bytes of intermediates each,
# and this many (X, out, K, stream) combinations per adjacency
PREPARED_LOOP_MAX_BYTES = 1 << 26
PREPARED_LOOPS_KEPT = 4


class GraphedPropagation:
    """The K-hop loop of propagate() captured once into a HIP graph, for
    repeated propagation over one adjacency at one feature shape (many feature
    sets, serving, hyper-parameter sweeps like the reference's tuning.py).

    It makes the whole loop -- pad copy, K SpMM launches, the hub kernels'
    fork/join on the side stream -- one replayable unit, e.g. inside a larger
    captured serving step.  It is not a speed-up on its own: even at Pubmed
    shape a hop is GPU-bound, and a replay measured 118 us against 122 us
    eager at K=2, the static-input copy included
    (profiles/r01_bench_small_v2.log).  run(X) copies X into the graph's static
    input and replays; the result is in self.out (bit-identical to
    propagate()).
    Capture builds the plan first (it synchronises) and warms the code
    objects on a side stream, as torch.cuda.graph requires."""

    def __init__(self, csr: DeviceCSR, shape, K: int, threshold=None, hub_threshold=None):
        n, F = shape
        if K < 1:
            raise ValueError("GraphedPropagation: K >= 1")
        self.csr, self.K = csr, int(K)
        self.x_in = torch.empty((n, F), dtype=torch.float32, device=csr.device)
        self.out = torch.empty((n, F), dtype=torch.float32, device=csr.device)
        self.x_in.zero_()
        kw = dict(threshold=threshold, hub_threshold=hub_threshold)
        csr.plan(0, n, threshold, hub_threshold, F)  # synchronous: never inside the capture
        side = torch.cuda.Stream(device=csr.device)
        side.wait_stream(torch.cuda.current_stream(csr.device))
        with torch.cuda.stream(side):  # (no launch list kept for the side stream)
            propagate(csr, self.x_in, self.K, out=self.out, prepare=False, **kw)
        torch.cuda.current_stream(csr.device).wait_stream(side)
        torch.cuda.synchronize(csr.device)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            propagate(csr, self.x_in, self.K, out=self.out, prepare=False, **kw)

    def run(self, X: torch.Tensor) -> torch.Tensor:
        X = _check_features(X, self.csr)
        if tuple(X.shape) != tuple(self.x_in.shape):
            raise RuntimeError(f"GraphedPropagation: captured for {tuple(self.x_in.shape)}, "
                               f"got {tuple(X.shape)}")
        self.x_in.copy_(X)
        self.graph.replay()
        return self.out


WARM_PROPAGATE, WARM_CLASSIFIER, WARM_LOADERS = 1, 2, 4  # sgc_warmup units (sgc_amd.h)
_warmed = {}


def warmup(device=None, units=WARM_PROPAGATE | WARM_CLASSIFIER):
    """Load the library's code objects on `device` now (sgc_warmup: one empty
    launch per translation unit), once per process and device, so that the
    first sgc_precompute a caller times (reddit.py:43,72-74) does not pay
    them.  The loaders call it when they move data to the GPU.  Returns the
    seconds it took (0.0 when already done)."""
    import time
    d = torch.device("cuda") if device is None else torch.device(device)
    dev = torch.device("cuda", d.index if d.index is not None else torch.cuda.current_device())
    key = (dev.index, int(units))
    if key in _warmed:
        return 0.0
    lib = _lib.load()
    t = time.perf_counter()
    with torch.cuda.device(dev):
        _lib.check(lib.sgc_warmup(int(units), _lib.stream_handle(dev)), "warmup")
        if units & WARM_PROPAGATE:
            # one tiny propagation through the same steps as sgc_precompute's
            # one-GPU path, so the torch kernels they use (COO accessors,
            # indexing, allocation) load here as well; the COO is row-unsorted
            # (the ingest's sort runs too).  No process-group step: under
            # torchrun every rank warms on its own.
            n = 64
            i = torch.arange(n, device=dev)
            idx = torch.stack([torch.cat([(i + 1) % n, i]), torch.cat([i, i])])
            adj = torch.sparse_coo_tensor(idx, torch.full((2 * n,), 0.5, device=dev), (n, n))
            csr = csr_of(adj)
            propagate(csr, torch.ones((n, 8), device=dev), 2)
            # the multi-GPU partitions' device-built shards (searchsorted,
            # indexing, casts): their torch kernels' first use cost the first
            # P = 4 call ~0.2 s of its 0.42 (profiles/r06/s20)
            from .distributed import _chunk_order, make_shard_device
            make_shard_device(csr, 1, 3)
            _chunk_order(csr, [(0, 32), (32, n)])
        torch.cuda.synchronize(dev)
        if units & WARM_PROPAGATE:
            # torch's stream pool for this device (the multi-GPU partitions'
            # chunk / tail streams): its first use creates the pool's streams,
            # new hardware queues among them (~8 ms each, profiles/r06/s10)
            torch.cuda.Stream(device=dev)
            # under torchrun: the process group the partitioned sgc_precompute
            # uses is set up here, with the loaders (rendezvous and RCCL's
            # communicator, eagerly bound to this device), not inside the
            # first call the reference times (reddit.py:43)
            from . import multigpu
            multigpu.process_group(dev)
    _warmed[key] = time.perf_counter() - t
    return _warmed[key]


def kernel_timing(on: bool):
    """Turn per-kernel launch timing on/off (sgc_timing_enable; diagnostics)."""
    _lib.check(_lib.load().sgc_timing_enable(1 if on else 0), "timing_enable")


def collect_kernel_timing(capacity=1 << 16):
    """(light_ms, hub_ms) lists of the SpMM launches recorded since the last
    collect; hub_ms[i] is None for a launch without hub rows (synchronous)."""
    import ctypes
    lib = _lib.load()
    light = (ctypes.c_float * capacity)()
    hub = (ctypes.c_float * capacity)()
    n = _lib._i64(0)
    _lib.check(lib.sgc_timing_collect(ctypes.cast(light, ctypes.c_void_p),
                                      ctypes.cast(hub, ctypes.c_void_p), capacity,
                                      ctypes_byref(n)), "timing_collect")
    k = int(n.value)
    return [float(light[i]) for i in range(k)], [float(hub[i]) if hub[i] >= 0 else None
                                                 for i in range(k)]


def collect_launch_timing(capacity=1 << 16):
    """Per SpMM launch since the last collect: (light_ms, hub_ms, span_ms,
    light_kernel) lists -- span = the whole launch as the caller's stream
    sees it (hub kernel joined); light_kernel = "spmm_csr_kernel",
    "spmm_rows_kernel" or None (a hub-only launch); hub_ms None without hub
    rows."""
    import ctypes
    lib = _lib.load()
    light = (ctypes.c_float * capacity)()
    hub = (ctypes.c_float * capacity)()
    span = (ctypes.c_float * capacity)()
    kind = (ctypes.c_int32 * capacity)()
    n = _lib._i64(0)
    _lib.check(lib.sgc_timing_collect_ex(*(ctypes.cast(b, ctypes.c_void_p)
                                           for b in (light, hub, span, kind)),
                                         capacity, ctypes_byref(n)), "timing_collect_ex")
    names = {0: "spmm_csr_kernel", 1: "spmm_rows_kernel", 2: "spmm_rows_kernel+hub (fused)",
             3: "spmm_csr_kernel+hub (fused)"}
    k = int(n.value)
    return ([float(light[i]) for i in range(k)],
            [float(hub[i]) if hub[i] >= 0 else None for i in range(k)],
            [float(span[i]) for i in range(k)],
            [names.get(int(kind[i])) for i in range(k)])


def linear(X: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None, out=None):
    """Y = X . W^T + b on fp32 MFMA (reference models.py:17-18, nn.Linear)."""
    _require_device(X, "input")
    if X.dtype != torch.float32 or weight.dtype != torch.float32:
        raise TypeError("sgc_amd.linear: float32 only")
    if X.dim() != 2:
        raise ValueError("sgc_amd.linear: 2-D input expected")
    M, K = X.shape
    C = weight.shape[0]
    if weight.shape[1] != K:
        raise RuntimeError(f"sgc_amd.linear: shape mismatch {tuple(X.shape)} x {tuple(weight.shape)}^T")
    if X.stride(1) != 1 or X.stride(0) < K:
        X = X.contiguous()
    W = weight.contiguous()
    b = bias.contiguous() if bias is not None else None
    if out is None:
        out = torch.empty((M, C), dtype=torch.float32, device=X.device)
    lib = _lib.load()
    with torch.cuda.device(X.device):
        _lib.check(lib.sgc_linear_f32(_lib.ptr(X), X.stride(0), _lib.ptr(W), _lib.ptr(b),
                                      _lib.ptr(out), out.stride(0), M, K, C,
                                      _lib.stream_handle(X.device)), "linear_f32")
    return out


def linear_backward(X: torch.Tensor, grad_out: torch.Tensor, want_bias=True):
    """(dW, db) of Y = X W^T + b for dY = grad_out: dW = dY^T X, db = sum_m dY
    (None unless want_bias), one read of X on fp32 MFMA
    (sgc_linear_backward_f32).  At most 64 classes."""
    _require_device(X, "input")
    M, K = X.shape
    C = grad_out.shape[1]
    if grad_out.shape[0] != M or X.dtype != torch.float32 or grad_out.dtype != torch.float32:
        raise RuntimeError("sgc_amd.linear_backward: shape/dtype mismatch")
    if C > 64:
        raise ValueError("sgc_amd.linear_backward: at most 64 classes")
    if X.stride(1) != 1 or X.stride(0) < K:
        X = X.contiguous()
    if grad_out.stride(1) != 1 or grad_out.stride(0) < C:
        grad_out = grad_out.contiguous()
    dW = torch.empty((C, K), dtype=torch.float32, device=X.device)
    db = torch.empty(C, dtype=torch.float32, device=X.device) if want_bias else None
    if M == 0:
        dW.zero_()
        if db is not None:
            db.zero_()
        return dW, db
    lib = _lib.load()
    ws_bytes = lib.sgc_linear_backward_workspace(M, K, C)
    ws = torch.empty(max(1, ws_bytes), dtype=torch.uint8, device=X.device)
    with torch.cuda.device(X.device):
        _lib.check(lib.sgc_linear_backward_f32(_lib.ptr(X), X.stride(0), _lib.ptr(grad_out),
                                               grad_out.stride(0), M, K, C, _lib.ptr(dW),
                                               _lib.ptr(db), _lib.ptr(ws), ws_bytes,
                                               _lib.stream_handle(X.device)), "linear_backward_f32")
    return dW, db


def linear_xent(X: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor],
                labels: torch.Tensor, want_logits=False):
    """Fused SGC training step: (loss, dW, db[, logits]) for
    F.cross_entropy(X W^T + b, labels) (mean), on the GPU (sgc_linear_xent_f32)."""
    _require_device(X, "input")
    if X.dtype != torch.float32 or weight.dtype != torch.float32:
        raise TypeError("sgc_amd.linear_xent: float32 only")
    M, K = X.shape
    C = weight.shape[0]
    if weight.shape[1] != K or labels.shape != (M,):
        raise RuntimeError("sgc_amd.linear_xent: shape mismatch")
    if C > 64:
        raise ValueError("sgc_amd.linear_xent: at most 64 classes")
    if X.stride(1) != 1 or X.stride(0) < K:
        X = X.contiguous()
    W = weight.detach().contiguous()
    b = bias.detach().contiguous() if bias is not None else None
    y = labels.to(device=X.device, dtype=torch.int64).contiguous()
    if M:
        # F.cross_entropy raises on a label outside [0, C) (and skips
        # ignore_index=-100 rows, which the fused kernel does not support):
        # refuse loudly instead of returning a silently different loss
        lo, hi = (int(v) for v in torch.aminmax(y))
        if lo < 0 or hi >= C:
            raise ValueError(f"sgc_amd.linear_xent: labels must lie in [0, {C}), got "
                             f"[{lo}, {hi}] (ignore_index is not supported)")
    lib = _lib.load()
    loss = torch.empty((), dtype=torch.float32, device=X.device)
    dW = torch.empty_like(W)
    db = torch.empty(C, dtype=torch.float32, device=X.device) if b is not None else None
    logits = torch.empty((M, C), dtype=torch.float32, device=X.device) if want_logits else None
    ws_bytes = lib.sgc_linear_xent_workspace(M, K, C)
    ws = torch.empty(max(1, ws_bytes), dtype=torch.uint8, device=X.device)
    with torch.cuda.device(X.device):
        _lib.check(lib.sgc_linear_xent_f32(_lib.ptr(X), X.stride(0), _lib.ptr(W), _lib.ptr(b),
                                           _lib.ptr(y), M, K, C, _lib.ptr(loss), _lib.ptr(dW),
                                           _lib.ptr(db), _lib.ptr(logits), C, _lib.ptr(ws),
                                           ws_bytes, _lib.stream_handle(X.device)),
                   "linear_xent_f32")
    return (loss, dW, db, logits) if want_logits else (loss, dW, db)
