"""Rehearse the PUBLIC multi-GPU call -- sgc_precompute with every rank getting
the whole X_K (reference reddit.py:43 -> utils.py:92-97) -- on ONE GPU.

    python scripts/replicated_rehearsal.py [--shape reddit] [--P 2,4,8]
                                           [--link-gbps 57.6] [--ranks all]

For each P and each candidate of the auto partition (sgc_amd.multigpu
AUTO_CANDIDATES: replicate / features / lines), every rank's exact step runs
through the product propagator with the collectives replaced by local copies
(the gather writes nothing: the rank's own slot is already in place, the
other slots hold zeros), so what is timed is the rank's compute: hops, the
last hop in row chunks written into the gather buffers' slots, the unpack
of every chunk into X_K (one block-copy launch per chunk), the line
partition's tail hops and gathers on their stream.

Measured, per rank and candidate:
  compute_replicated_ms / compute_sharded_ms  the whole step, replicated and
      sharded output (the difference is the replication's local work);
  chunk_ready_ms  when each last-hop chunk's rows are done (events), the run
      repeated with a concurrent copy of the gather's bytes on a second
      stream from the first chunk's readiness on ((P-1)/P of X_K read and
      written: the HBM traffic RCCL's all-gathers add on a rank, here all at
      HBM speed rather than spread over the link time) -- the compute
      timeline under that interference is the one the projection uses;
  unpack_ms  one chunk's block-copy launch;
  breakdown (--breakdown)  the replicated step with the final unpacks
      skipped, and with the last hop in one chunk (with and without the
      unpacks): compute_replicated - compute_sharded split into the unpack,
      the chunking and the rest.
Modelled at a STATED link rate (one xGMI link per GPU pair, --link-gbps each
way, a rank's ingress (P-1) links):
  chunk c's all-gather ((P-1) blocks of its rows) starts when the chunk is
  ready (measured, under the concurrent copy) and the previous gather is
  done, takes its bytes / ingress; the step ends at max(compute end, last
  gather end + one unpack); the line partition's per-hop tail gathers add
  what their hop's main launch does not cover.  "replicate" is one GPU's
  measured time.  One JSON line per rank and candidate, a summary per P.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sgc_amd import graphs  # noqa: E402
from sgc_amd.distributed import (IPC_DONE, IPC_FLAG_WORDS,  # noqa: E402
                                 FeaturePartitionedPropagator, IpcPeers,
                                 LinePartitionedPropagator, _copy_blocks, feature_bounds,
                                 line_bounds, make_shard, replicated_chunks)
from sgc_amd.propagate import DeviceCSR, propagate  # noqa: E402


class _Local:
    """Collectives replaced by local no-ops (slots already in place); each
    main-gather call records an event on the current stream: the moment its
    chunk's rows are done."""

    side_copy = None  # (stream, src, dst): started at the first mark

    def _reset_marks(self):
        self.marks = []
        if getattr(self, "_ipc", None) is not None:
            self._ipc._marks = self.marks

    def _mark(self, dst):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        if not self.marks and self.side_copy is not None:
            # the gathers' HBM traffic starts with the first gather
            side, a, b = self.side_copy
            side.wait_event(ev)
            with torch.cuda.stream(side):
                b.copy_(a)
        self.marks.append((ev, dst.shape[0]))


class LocalFeatures(_Local, FeaturePartitionedPropagator):
    def _all_gather(self, full, loc):
        self._mark(full)
        return None

    def _all_to_all(self, recv, send):
        recv.copy_(send)
        return None

    def _exchange_pair(self, send, dst, recv, src):
        m = min(send.shape[0], recv.shape[0])
        if m:
            recv[:m].copy_(send[:m])
        return []


class LocalIpcPeers(IpcPeers):
    """The IPC window of a rehearsed rank: every "peer" maps to this rank's
    own window (pulls read P blocks at local HBM speed: on a node the P - 1
    peer blocks come over the links, their reads land on the peers' HBM and
    the pulls' writes on this rank's); chunk flags record a timing event (the
    chunk's readiness) when raised."""

    def __init__(self, rank, world, n, ld, device, marks):
        self.rank, self.world, self.n, self.ld = rank, world, int(n), int(ld)
        half = self.n * self.ld
        self.window = torch.zeros(2 * half + IPC_FLAG_WORDS, dtype=torch.float32, device=device)
        self.flags = self.window[2 * half:].view(torch.int32)
        self.halves = [self.window[:half].view(self.n, self.ld),
                       self.window[half:2 * half].view(self.n, self.ld)]
        self.err = torch.zeros(1, dtype=torch.int32).pin_memory()
        self.ptrs = [self.window.data_ptr()] * world
        self._bases = []
        self.seq = 0
        self._marks = marks

    def signal(self, word, value, stream):
        super().signal(word, value, stream)
        if word < IPC_DONE:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(stream)
            self._marks.append((ev, 0))


def _ipc_rehearsal(enable):
    """Route the feature / line partitions' replicated last hop through
    LocalIpcPeers (enable) or through the collective path (not)."""
    import sgc_amd.distributed as D
    if not enable:
        os.environ["SGC_AMD_REPLICATED_EXCHANGE"] = "collective"
        return
    os.environ["SGC_AMD_REPLICATED_EXCHANGE"] = "ipc"

    def fake(prop, group, rank, world, n, ld, device):
        key = (n, ld, str(device))
        if getattr(prop, "_ipc_key", None) != key:
            prop._ipc = LocalIpcPeers(rank, world, n, ld, device, prop.marks)
            prop._ipc_key = key
        prop._ipc._marks = prop.marks
        return prop._ipc
    D._ipc_for = fake


class LocalLines(_Local, LinePartitionedPropagator):
    def _collective(self, kind, dst, src):
        if kind == "gather" and dst.shape[1] != self._tail_ld:
            self._mark(dst)
        elif kind != "gather":
            m = min(src.shape[0], dst.shape[0])
            dst[:m].copy_(src[:m])
        return None


def _buffers_zero(prop):
    for b in prop._bufs.values():
        b.zero_()


def timeit(fn, reps, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return float(np.median(ts))


def timeline(prop, X0, K, reps, copy=None):
    """Median (step ms, [chunk ready ms]) of the replicated step; `copy` =
    (src, dst) copied on a second stream from the moment the first chunk is
    ready (when the first gather, and with it RCCL's traffic, starts)."""
    side = torch.cuda.Stream()
    steps, readies = [], []
    prop.side_copy = None if copy is None else (side, copy[0], copy[1])
    for r in range(reps + 1):
        prop._reset_marks()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        prop.propagate(X0, K, output="replicated")
        e.record()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        if r == 0:
            continue  # warm-up
        steps.append(s.elapsed_time(e))
        readies.append([s.elapsed_time(ev) for ev, _ in prop.marks])
    prop.side_copy = None
    return float(np.median(steps)), [float(v) for v in np.median(np.array(readies), axis=0)]


def breakdown(prop, X0, K, reps):
    """The replicated step (a) with the unpacks of the gather buffers into
    X_K skipped, (b) with the last hop in one chunk, (c) both."""
    import sgc_amd.distributed as D
    real = D._copy_blocks
    fulls = {b.data_ptr() for k, b in prop._bufs.items() if k[0] == "full"}

    def no_unpack(src, dst, segs):
        if src.data_ptr() not in fulls:
            real(src, dst, segs)

    run = lambda: prop.propagate(X0, K, output="replicated")  # noqa: E731
    res = {}
    chunks = prop.chunks
    for name, c, skip in (("no_unpack", chunks, True), ("one_chunk", 1, False),
                          ("one_chunk_no_unpack", 1, True)):
        prop.chunks = c
        D._copy_blocks = no_unpack if skip else real
        try:
            run()
            torch.cuda.synchronize()
            fulls |= {b.data_ptr() for k, b in prop._bufs.items() if k[0] == "full"}
            res[name] = timeit(run, reps)
        finally:
            D._copy_blocks = real
            prop.chunks = chunks
    return res


def project(step_ms, ready_ms, gather_bytes, unpack_ms, ingress):
    end = 0.0
    for t, nb in zip(ready_ms, gather_bytes):
        end = max(end, t) + nb / ingress * 1e3
    return max(step_ms, end + unpack_ms)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="reddit")
    ap.add_argument("--P", default="2,4,8")
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--ranks", default="all")
    ap.add_argument("--link-gbps", type=float, default=57.6,
                    help="per-peer xGMI rate each way (one link per GPU pair)")
    ap.add_argument("--schedules", default="",
                    help="';'-separated knob sets of the last hop's chunk schedule, e.g. "
                         "'alone=0,hub=0;alone=1,hub=1' (sgc_amd.distributed "
                         "FIRST_CHUNK_ALONE / HUB_EARLY); default: the product's")
    ap.add_argument("--breakdown", action="store_true",
                    help="time the replicated step without unpacks / in one chunk too")
    ap.add_argument("--fractions", default="",
                    help="semicolon-separated row fractions of the last hop's chunks to "
                         "compare, e.g. 1,3,3,1;1,1,2,3,1 (sgc_amd.distributed.REPLICATED_CHUNKS)")
    ap.add_argument("--exchange", default="ipc", choices=["ipc", "collective"],
                    help="the replicated last hop: IPC pulls of the peers' blocks straight "
                         "into X_K (the product's default on a GPU node) or in-place "
                         "all-gathers + unpack")
    ap.add_argument("--chunks", type=int, default=4,
                    help="last-hop chunks (4 = the product's 1:3:3:1 split, else equal)")
    args = ap.parse_args()
    _ipc_rehearsal(args.exchange == "ipc")
    spec = graphs.SHAPES[args.shape]
    S = graphs.synthetic_graph(args.shape, seed=0)
    F, K, n = spec["features"], spec["hops"], S.n
    X0 = torch.from_numpy(graphs.synthetic_features(args.shape, n, F, seed=1)).cuda()
    csr = DeviceCSR.from_host_arrays(S.row_ptr, S.col_idx, S.val, device="cuda")
    out = torch.empty((n, F), device="cuda")
    t1 = timeit(lambda: propagate(csr, X0, K, out=out), args.reps)
    print(json.dumps({"case": "single", "shape": args.shape, "ms": t1}), flush=True)
    import sgc_amd.distributed as D
    scheds = [dict(kv.split("=") for kv in part.split(",") if kv)
              for part in args.schedules.split(";")] if args.schedules else [{}]
    fracs = ([tuple(int(v) for v in part.split(",")) for part in args.fractions.split(";")]
             if args.fractions else [D.REPLICATED_CHUNKS])
    for fr in fracs:
        D.REPLICATED_CHUNKS = fr
        for sched in scheds:
            D.FIRST_CHUNK_ALONE = bool(int(sched.get("alone", int(D.FIRST_CHUNK_ALONE))))
            D.HUB_EARLY = bool(int(sched.get("hub", int(D.HUB_EARLY))))
            D.CHUNK_STREAMS = int(sched.get("streams", D.CHUNK_STREAMS))
            run_schedule(args, S, csr, X0, out, t1, F, K, n,
                         {"alone": int(D.FIRST_CHUNK_ALONE), "hub": int(D.HUB_EARLY),
                          "streams": D.CHUNK_STREAMS, "fractions": list(fr)})


def run_schedule(args, S, csr, X0, out, t1, F, K, n, sched):
    for P in (int(v) for v in args.P.split(",")):
        ingress = (P - 1) * args.link_gbps * 1e9
        best = {"replicate": t1}
        rank_recs = {}
        sel = range(P) if args.ranks == "all" else [int(r) for r in args.ranks.split(",")]
        for cand in ("features", "lines"):
            recs = []
            for p in sel:
                if cand == "features":
                    prop = LocalFeatures(csr, rank=p, world_size=P, chunks=args.chunks)
                    bounds, B = feature_bounds(F, P)
                    wcols = B
                else:
                    W, T = line_bounds(F, P)
                    if W == 0:
                        break
                    shard = make_shard(S.row_ptr, S.col_idx, S.val, p, P, "cuda")
                    prop = LocalLines(shard, csr=csr, chunks=args.chunks)
                    prop._tail_ld = (max(F - T, 1) + 31) // 32 * 32
                    wcols = W
                prop._reset_marks()
                prop.propagate(X0, K, output="replicated")  # allocate the buffers
                torch.cuda.synchronize()
                _buffers_zero(prop)
                t_rep = timeit(lambda: prop.propagate(X0, K, output="replicated"), args.reps)
                t_sh = timeit(lambda: prop.propagate(X0, K, output="sharded"), args.reps)
                # the chunk timeline alone and under a concurrent copy of the
                # gather's bytes ((P-1)/P of X_K, read + written)
                step0, ready0 = timeline(prop, X0, K, args.reps)
                import sgc_amd.distributed as D
                chunks = replicated_chunks(n, D.REPLICATED_CHUNKS if prop.chunks == 4
                                           else (1,) * prop.chunks)
                gbytes = [(P - 1) * (r1 - r0) * wcols * 4 for r0, r1 in chunks]
                if args.exchange == "ipc":
                    # the pulls are in the step (P blocks read at local HBM
                    # speed and written into X_K): no side copy, no unpack
                    step1, ready1, t_unpack = step0, ready0, 0.0
                else:
                    nb = int((P - 1) / P * n * F)
                    src = torch.empty(nb, device="cuda")
                    dst = torch.empty(nb, device="cuda")
                    step1, ready1 = timeline(prop, X0, K, args.reps, copy=(src, dst))
                    del src, dst
                    # one chunk's unpack (the block-copy launch of P blocks)
                    r0, r1 = chunks[-1]
                    rows = r1 - r0
                    full = prop._bufs[("full", len(chunks) - 1)]
                    cb = [(q * rows, 0, r0, min(q * wcols, F), rows,
                           min((q + 1) * wcols, F) - min(q * wcols, F)) for q in range(P)]
                    t_unpack = timeit(lambda: _copy_blocks(full, out, cb), args.reps)
                tail_exposed = 0.0
                if cand == "lines" and F - line_bounds(F, P)[1] > 0:
                    # each hop's tail gather beside that hop's main launch
                    # (round-4 model): what a main hop (~ step / K) does not cover
                    tb = (P - 1) * shard.block * prop._tail_ld * 4
                    tail_exposed = K * max(0.0, tb / ingress * 1e3 - step0 / (K + 1))
                proj = project(step1, ready1, gbytes, t_unpack, ingress) + tail_exposed
                bd = breakdown(prop, X0, K, args.reps) if (args.breakdown and
                                                            args.exchange == "collective") else None
                rec = {"case": "rank", "schedule": sched, "exchange": args.exchange, "P": P,
                       "candidate": cand, "rank": p,
                       "block_cols": wcols, "compute_replicated_ms": t_rep,
                       "compute_sharded_ms": t_sh, "replication_local_ms": t_rep - t_sh,
                       "step_ms": step0, "chunk_ready_ms": ready0,
                       "step_with_copy_ms": step1, "chunk_ready_with_copy_ms": ready1,
                       "gather_MB": [round(v / 1e6, 1) for v in gbytes],
                       "gather_ms": [v / ingress * 1e3 for v in gbytes],
                       "unpack_ms": t_unpack, "tail_exposed_ms": tail_exposed,
                       "projected_replicated_ms": proj}
                if bd is not None:
                    rec["breakdown_ms"] = dict(bd, sharded=t_sh, replicated=t_rep)
                print(json.dumps(rec), flush=True)
                recs.append(rec)
                del prop
                torch.cuda.empty_cache()
            if recs:
                best[cand] = max(r["projected_replicated_ms"] for r in recs)
                rank_recs[cand] = recs
        chosen = min(best, key=best.get)
        summ = {"case": "summary", "schedule": sched, "exchange": args.exchange, "P": P,
                "single_ms": t1, "link_GBps_each_way": args.link_gbps,
                "projected_ms": best, "projected_speedup": {c: t1 / v for c, v in best.items()},
                "auto_would_choose": chosen, "auto_speedup": t1 / best[chosen],
                "replication_local_ms_max": {c: max(r["replication_local_ms"] for r in rs)
                                             for c, rs in rank_recs.items()},
                "assumption": "one xGMI link per GPU pair at link_GBps each way; compute "
                              "measured on one GPU per rank, the last hop's chunk timeline "
                              "under a concurrent copy of the gather's bytes; each chunk "
                              "gathered when ready, one unpack after the last"}
        print(json.dumps(summ), flush=True)


if __name__ == "__main__":
    main()
