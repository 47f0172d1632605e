"""sgc_precompute across GPUs behind the reference's own call.

The reference's drivers call `sgc_precompute(features, adj, degree)`
(reddit.py:43, citation.py:32 -> utils.py:92-97) and expect the whole X_K
back.  This module lets that unchanged call use every GPU of the node, in
either of two ways:

* one process per GPU (`torchrun --nproc-per-node N reddit.py`): importing
  the drop-in binds each process to cuda:LOCAL_RANK, so the caller's
  `.cuda()` tensors land on its own GPU; on the first sgc_precompute a process
  group is initialised from torchrun's environment (RCCL over xGMI when every
  local rank has a GPU of its own, gloo when ranks share one -- the host-staged
  rehearsal), or the caller's own initialised default group is used.  The K
  hops then run partitioned (sgc_amd.distributed) and every rank gets the
  full X_K, as the reference returns it;
* one process, several devices (`SGC_AMD_DEVICES=all` or `=0,1,2,3`): the
  native multi-device engine of the C ABI (sgc_mgpu_*, csrc/mgpu.hip) drives
  all of them from the single call; see `DeviceSet`.

Partition (SGC_AMD_PARTITION): "auto" (default) -- chosen by measured time:
the first call on an adjacency (per group, feature width and K) runs every
candidate of AUTO_CANDIDATES once to warm it and once timed, takes the
slowest rank's time of each (one all-reduce), keeps the fastest for every
later call and returns its X_K (all candidates give the same bits), so the
replicated call is never slower than one GPU's: "replicate" is a candidate;
"replicate" -- every rank computes all of X_K itself (no exchange; one GPU's
time at any P); "features" -- each rank runs all K hops over the whole S on
its block of feature columns, so the only exchange is one all-gather of X_K,
the least any partitioned replicated output can move; "lines" -- each rank
owns whole 128-B lines of features plus a row block of the leftover lines,
gathered after each hop (per-rank compute at Reddit shape, one GPU per rank:
P = 4 2.44 vs 3.03 ms, P = 8 1.52 vs 1.62; P = 2 5.44 vs 5.19, DESIGN.md
6.3); "rows" (nnz-balanced row blocks, an all-gather of X_k per hop: the
north star's 1-D row slicing) or "cyclic" (row tiles round-robin,
column-ordered exchange).
Every partition keeps each output element's FMA chain whole and in CSR
order, so X_K is bit-identical to one GPU's and to the reference.
"""
import os
import time

import torch
import torch.distributed as dist

PARTITIONS = ("auto", "tune", "replicate", "features", "lines", "rows", "cyclic")
# what "tune" times (the row and cyclic partitions move X_k after every hop:
# never faster for a replicated X_K)
AUTO_CANDIDATES = ("replicate", "features", "lines")
# below this much work (nnz(S) * F multiply-adds per hop) a call is a few
# hundred microseconds on one GPU and the exchange's latency would eat any
# split: "auto" replicates.  Pubmed shape: 5.4e7; Reddit shape: 1.4e10.
AUTO_MIN_WORK = 1 << 30


def torchrun_env():
    """(rank, world, local_rank, local_world) when launched by torchrun with
    more than one process, else None."""
    try:
        world = int(os.environ["WORLD_SIZE"])
        rank = int(os.environ["RANK"])
    except (KeyError, ValueError):
        return None
    if world <= 1:
        return None
    local = int(os.environ.get("LOCAL_RANK", rank))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world))
    return rank, world, local, local_world


def bind_local_device():
    """Under torchrun, make `cuda` mean cuda:(LOCAL_RANK mod visible GPUs) for
    this process, so an unchanged driver's `.cuda()` calls land on its own
    GPU.  No-op without torchrun, without a GPU, or with
    SGC_AMD_BIND_DEVICE=0.  Returns the device index bound (or None)."""
    env = torchrun_env()
    if env is None or os.environ.get("SGC_AMD_BIND_DEVICE", "1") == "0":
        return None
    n = torch.cuda.device_count()  # does not initialise the runtime
    if n == 0:
        return None
    d = env[2] % n
    torch.cuda.set_device(d)
    return d


def process_group(device):
    """The group sgc_precompute partitions over, or None (one device).

    An initialised default group with world > 1 is used as is.  Under
    torchrun without one, it is initialised here (env://): backend
    SGC_AMD_DIST_BACKEND, else "nccl" (RCCL) when every local rank has a GPU of
    its own and the tensors are on the GPU, else "gloo".
    SGC_AMD_AUTO_DIST=0 turns the whole multi-process mode off."""
    if os.environ.get("SGC_AMD_AUTO_DIST", "1") == "0" or not dist.is_available():
        return None
    if dist.is_initialized():
        return dist.group.WORLD if dist.get_world_size() > 1 else None
    env = torchrun_env()
    if env is None:
        return None
    backend = os.environ.get("SGC_AMD_DIST_BACKEND")
    if not backend:
        own_gpu = device.type == "cuda" and torch.cuda.device_count() >= env[3]
        backend = "nccl" if own_gpu else "gloo"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=device)
    else:
        dist.init_process_group(backend)
    return dist.group.WORLD


def partition_name(world=None):
    """The partition SGC_AMD_PARTITION names ("auto", the default: a persisted
    per-node choice when one exists, else rule_choice -- one propagation on
    the first call, no trials; "tune": the same first call, candidates timed
    on the second; precompute_group).  `world` is accepted for the callers
    that pass it; it does not change the name."""
    p = os.environ.get("SGC_AMD_PARTITION", "auto")
    if p not in PARTITIONS:
        raise ValueError(f"SGC_AMD_PARTITION must be one of {PARTITIONS}, not {p!r}")
    return p


def rule_choice(world, n, nnz, F, K):
    """The partition "auto" uses without a persisted choice, from the one-GPU
    rehearsal of every candidate at Reddit shape: at P = 2
    replicating beats both splits (the one link carries half of X_K: features
    0.95-0.97x, lines 0.88-0.92x), at P >= 3 the line partition leads (P = 4
    1.85x, P = 8 2.8-3.1x; features 1.6x / 2.8-2.9x), provided each rank owns
    at least one whole 128-B line (F >= 32 P), else features; calls with less
    than AUTO_MIN_WORK multiply-adds per hop replicate (they are latency-bound
    on one GPU).  Identical on every rank: no collective."""
    min_work = int(os.environ.get("SGC_AMD_AUTO_MIN_WORK", AUTO_MIN_WORK))
    if world <= 2 or K <= 0 or int(nnz) * int(F) < min_work:
        return "replicate"
    from .distributed import line_bounds
    W, _ = line_bounds(int(F), int(world))
    return "lines" if W > 0 else "features"


def _lib_sha():
    """sha256 of the loaded libsgc_amd.so (part of a persisted choice's key:
    a new library may change which candidate wins)."""
    import hashlib
    from . import _lib
    h = hashlib.sha256()
    with open(_lib.LIB_PATH, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def tune_file():
    """Where "tune" persists its measured choices (one JSON object per node):
    SGC_AMD_TUNE_FILE, default ~/.cache/sgc_amd/partitions.json."""
    return os.environ.get("SGC_AMD_TUNE_FILE") or os.path.join(
        os.path.expanduser("~"), ".cache", "sgc_amd", "partitions.json")


def _tune_key(world, n, nnz, F, K, device):
    name = torch.cuda.get_device_name(device) if device.type == "cuda" else "cpu"
    return f"world={world} n={n} nnz={nnz} F={F} K={K} dev={name} lib={_lib_sha()[:16]}"


def persisted_choice(world, n, nnz, F, K, device):
    """A choice "tune" measured earlier on this node for exactly this
    (world, n, nnz, F, K, device model, library), or None."""
    path = tune_file()
    if not os.path.exists(path):
        return None
    import json
    try:
        with open(path) as f:
            rec = json.load(f).get(_tune_key(world, n, nnz, F, K, device))
    except (OSError, ValueError):
        return None
    c = rec.get("chosen") if isinstance(rec, dict) else None
    return c if c in AUTO_CANDIDATES else None


def _persist_choice(world, n, nnz, F, K, device, chosen, seconds):
    import json
    path = tune_file()
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            d = {}
        d[_tune_key(world, n, nnz, F, K, device)] = {"chosen": chosen, "seconds": seconds}
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "w") as f:
            json.dump(d, f, indent=1, sort_keys=True)
        os.replace(tmp, path)
    except OSError:
        pass  # a read-only home: the choice is kept for this process only


def _host_csr(csr):
    """Host copies (numpy) of a DeviceCSR's arrays, cached on it: the row and
    cyclic partitions slice S on the host once per adjacency."""
    key = ("host_arrays",)
    if key not in csr._plans:
        csr._plans[key] = tuple(t.cpu().numpy() for t in (csr.row_ptr, csr.col_idx, csr.val))
    return csr._plans[key]


def _propagator(csr, group, partition, staging):
    """The partitioned propagator for (adjacency, group, partition), built once
    and cached on the adjacency's CSR with its buffers and prepared launches."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    key = ("dist", id(group), rank, world, partition, staging)
    prop = csr._plans.get(key)
    if prop is not None:
        return prop
    from .distributed import setup_stage
    with setup_stage(f"build_{partition}", csr.device):
        prop = _build_propagator(csr, group, partition, staging, rank, world)
    csr._plans[key] = prop
    return prop


def _build_propagator(csr, group, partition, staging, rank, world):
    from .distributed import (CyclicRowPropagator, FeaturePartitionedPropagator,
                              LinePartitionedPropagator, RowPartitionedPropagator,
                              make_shard_device)
    if partition == "replicate":
        prop = ReplicatedPropagator(csr)
    elif partition == "features":
        prop = FeaturePartitionedPropagator(csr, rank=rank, world_size=world, group=group,
                                            host_staging=staging)
    elif partition == "lines":
        shard = make_shard_device(csr, rank, world)  # no host copy of S
        prop = LinePartitionedPropagator(shard, csr=csr, group=group, host_staging=staging)
    elif partition == "rows":
        shard = make_shard_device(csr, rank, world)
        prop = RowPartitionedPropagator(shard, group=group, host_staging=staging)
    else:
        rp, ci, va = _host_csr(csr)
        groups = 1 if world <= 2 else 2 if world <= 4 else 3
        prop = CyclicRowPropagator(rp, ci, va, rank, world, csr.device, group=group,
                                   groups=groups, host_staging=staging)
    return prop


class ReplicatedPropagator:
    """Every rank computes all of X_K itself: the single-GPU propagation, no
    exchange -- one GPU's time at any world size, the floor the partitioned
    candidates must beat for a replicated X_K."""

    def __init__(self, csr):
        self.csr = csr

    def propagate(self, X0, K, out=None, output="replicated"):
        if output != "replicated":
            raise ValueError("ReplicatedPropagator: output='replicated' only")
        from .propagate import propagate
        return propagate(self.csr, X0, K, out=out)


def _sync(X):
    if X.is_cuda:
        torch.cuda.synchronize(X.device)


def _align(X, group):
    """A barrier through the group's own backend on X's device (a one-float
    all-reduce, then a synchronise): no device guess as dist.barrier makes."""
    dev = X.device if dist.get_backend(group) == "nccl" else torch.device("cpu")
    t = torch.zeros(1, device=dev)
    dist.all_reduce(t, group=group)
    _sync(X)


def _slowest(seconds, X, group):
    """Max over the group's ranks of each rank's seconds (list), one all-reduce."""
    dev = X.device if dist.get_backend(group) == "nccl" else torch.device("cpu")
    t = torch.tensor(seconds, dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return [float(v) for v in t.cpu()]


def auto_choice(csr, group, F, K):
    """The auto partition's record for (adjacency, group, F, K) once chosen:
    {"chosen": name, "how": "rule" | "persisted" | "timed", "seconds":
    {candidate: slowest rank's time} (timed only)}, or None."""
    return csr._plans.get(("auto", id(group), dist.get_world_size(group), int(F), int(K)))


# how many partitioned propagations precompute_group ran (tests: the first
# call of "auto" / "tune" runs exactly one)
PROPAGATIONS = [0]


def _run(prop, X, K):
    PROPAGATIONS[0] += 1
    from .distributed import setup_stage
    with setup_stage(f"propagate_{PROPAGATIONS[0]}", X.device):
        return prop.propagate(X, K, output="replicated")


def _drop_propagator(csr, group, name, staging):
    """Forget a candidate's propagator and its buffers (a tuned loser)."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    prop = csr._plans.pop(("dist", id(group), rank, world, name, staging), None)
    if prop is not None and hasattr(prop, "release"):
        prop.release()


def precompute_group(csr, X, K, group):
    """X_K = S^K X on every rank of `group`, partitioned (the caller has
    checked shapes and devices).  Collective: every rank must call it with
    the same adjacency and feature shape.

    "auto" (default): the first call runs ONE partition -- a choice "tune"
    persisted for this node and (world, n, nnz, F, K, library), broadcast
    from rank 0, else rule_choice (no collective) -- so the call the
    reference times (reddit.py:43, made once per adjacency) pays no trials.
    "tune": the same first call; the second call times every candidate (a
    warm and a timed call each, the slowest rank's time by one all-reduce),
    keeps the fastest for later calls, persists it (tune_file()) and frees the
    others' propagators."""
    staging = X.is_cuda and dist.get_backend(group) != "nccl"
    name = partition_name()
    if name not in ("auto", "tune"):
        return _run(_propagator(csr, group, name, staging), X, K)
    world = dist.get_world_size(group)
    n, F = int(X.shape[0]), int(X.shape[1])
    key = ("auto", id(group), world, F, int(K))
    rec = csr._plans.get(key)
    if rec is None:
        chosen, how = None, "rule"
        per = persisted_choice(world, n, csr.nnz, F, K, X.device)
        if per is not None or name == "tune":
            # agree on rank 0's file (ranks of several nodes may see others)
            idx = torch.tensor([AUTO_CANDIDATES.index(per) if per else -1], dtype=torch.int64,
                               device=X.device if dist.get_backend(group) == "nccl" else "cpu")
            dist.broadcast(idx, dist.get_global_rank(group, 0), group=group)
            if int(idx.item()) >= 0:
                chosen, how = AUTO_CANDIDATES[int(idx.item())], "persisted"
        if chosen is None:
            chosen = rule_choice(world, n, csr.nnz, F, K)
        rec = csr._plans[key] = {"chosen": chosen, "how": how, "seconds": None, "calls": 0}
    rec["calls"] += 1
    if name == "tune" and rec["how"] == "rule" and rec["calls"] == 2:
        return _tune(csr, X, K, group, staging, rec)
    return _run(_propagator(csr, group, rec["chosen"], staging), X, K)


def _tune(csr, X, K, group, staging, rec):
    """Time every candidate (warm + timed call each; the slowest rank's time),
    keep and persist the fastest, free the rest; returns its X_K."""
    world = dist.get_world_size(group)
    cands = list(AUTO_CANDIDATES)
    secs = []
    for c in cands:
        prop = _propagator(csr, group, c, staging)
        _run(prop, X, K)
        _align(X, group)  # every rank starts the timed call together
        t0 = time.perf_counter()
        out = _run(prop, X, K)
        _sync(X)
        secs.append(time.perf_counter() - t0)
        del out  # never three X_K alive at once
    slow = _slowest(secs, X, group)
    best = min(range(len(cands)), key=lambda i: (slow[i], i))
    rec.update(chosen=cands[best], how="timed", seconds=dict(zip(cands, slow)))
    for c in cands:
        if c != rec["chosen"]:
            _drop_propagator(csr, group, c, staging)
    if dist.get_rank(group) == 0:
        _persist_choice(world, int(X.shape[0]), csr.nnz, int(X.shape[1]), K, X.device,
                        rec["chosen"], rec["seconds"])
    # the winner's result (every candidate's X_K is the same bits)
    return _run(_propagator(csr, group, rec["chosen"], staging), X, K)


# ---------------------------------------------------------------------------
# One process, several devices: the native engine (sgc_mgpu_*).

def devices_from_env(home):
    """Devices named by SGC_AMD_DEVICES ("all", or a comma list of indices;
    the list may repeat an index: virtual devices sharing a GPU, used to
    rehearse the engine on one GPU), with the caller's device `home` first.
    None when unset or naming a single device."""
    spec = os.environ.get("SGC_AMD_DEVICES", "").strip()
    if not spec:
        return None
    if spec == "all":
        devs = list(range(torch.cuda.device_count()))
    else:
        devs = [int(x) for x in spec.split(",") if x.strip()]
    if home in devs:
        devs.remove(home)
    devs = [home] + devs
    return devs if len(devs) > 1 else None


class DeviceSet:
    """The native multi-device engine for one ordered device list
    (csrc/mgpu.hip): sgc_mgpu_init once per process, one attached replica set
    per adjacency (cached on its DeviceCSR, detached when that is freed)."""

    _current = None
    _generation = 0

    def __init__(self, devices):
        from . import _lib
        import ctypes
        self.devices = list(devices)
        arr = (ctypes.c_int * len(self.devices))(*self.devices)
        _lib.check(_lib.load().sgc_mgpu_init(len(self.devices), ctypes.cast(arr, ctypes.c_void_p)),
                   "mgpu_init")
        DeviceSet._generation += 1
        self.generation = DeviceSet._generation  # handles of an earlier engine are void

    @classmethod
    def get(cls, devices):
        cur = cls._current
        if cur is None or cur.devices != list(devices):
            if cur is not None:
                cur.finalize()
            cls._current = cur = cls(devices)
        return cur

    def finalize(self):
        from . import _lib
        _lib.check(_lib.load().sgc_mgpu_finalize(), "mgpu_finalize")
        if DeviceSet._current is self:
            DeviceSet._current = None

    def attach(self, csr):
        """Handle of csr's replicas on every device (made once: one copy of S
        per device, plus its launch plans)."""
        import weakref
        from . import _lib
        key = ("mgpu", self.generation)
        h = csr._plans.get(key)
        if h is None:
            lib = _lib.load()
            out = _lib._i64(0)
            with torch.cuda.device(csr.device):
                _lib.check(lib.sgc_mgpu_attach(_lib.ptr(csr.row_ptr), _lib.ptr(csr.col_idx),
                                               _lib.ptr(csr.val), csr.n_rows, csr.nnz,
                                               _lib.stream_handle(csr.device),
                                               _ctypes_byref(out)), "mgpu_attach")
            h = int(out.value)
            csr._plans[key] = h
            weakref.finalize(csr, _detach, h)
        return h

    def propagate(self, csr, X, K, out):
        from . import _lib
        h = self.attach(csr)
        with torch.cuda.device(X.device):
            _lib.check(_lib.load().sgc_mgpu_propagate(h, _lib.ptr(X), X.stride(0), _lib.ptr(out),
                                                      out.stride(0), X.shape[1], int(K),
                                                      _lib.stream_handle(X.device)),
                       "mgpu_propagate")
        return out


def _ctypes_byref(x):
    import ctypes
    return ctypes.byref(x)


def _detach(handle):
    try:
        from . import _lib
        _lib.load().sgc_mgpu_detach(handle)
    except Exception:  # interpreter shutdown: the engine is gone with the process
        pass


def precompute_devices(csr, X, K, devices):
    """X_K on the caller's device, computed by the devices in `devices`
    (devices[0] = X's device) through the native engine."""
    n, F = X.shape
    out = torch.empty((n, F), dtype=torch.float32, device=X.device)
    if n == 0 or F == 0:
        return out
    return DeviceSet.get(devices).propagate(csr, X, K, out)


def feature_blocks(F, parts, align=4):
    """Column blocks of the feature partition (the same rule as
    sgc_amd.distributed.feature_bounds, which the native engine mirrors)."""
    from .distributed import feature_bounds
    b, _ = feature_bounds(F, parts, align)
    return [(int(b[i]), int(b[i + 1])) for i in range(parts)]


__all__ = ["torchrun_env", "bind_local_device", "process_group", "precompute_group",
           "devices_from_env", "DeviceSet", "precompute_devices", "feature_blocks",
           "PARTITIONS", "AUTO_CANDIDATES", "ReplicatedPropagator", "auto_choice",
           "rule_choice", "persisted_choice", "tune_file"]
