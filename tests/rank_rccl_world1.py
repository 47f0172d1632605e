"""Helper run by tests/test_gpu_multigpu.py (not a test module): the RCCL
calls of the partitioned propagators, on a one-GPU box.

    python tests/rank_rccl_world1.py [n]

RCCL refuses two ranks on one GPU ("Duplicate GPU detected",
profiles/r05/rccl_probe.log), so the P > 1 RCCL paths cannot run here.  This
script initialises a ONE-rank nccl (RCCL) group and sets the propagators'
`force_collectives` hook, which turns off their one-rank shortcuts: the
exchange then goes through RCCL exactly as at P > 1 -- the feature and line
partitions' last hop in row chunks written into their slot of each chunk's
gather buffer and all-gathered IN PLACE (async), the waits on the compute
stream, the block-copy unpack -- and X_K must equal one GPU's bit for bit.
Then the line partition's tail-stream pattern itself: an async all_gather
issued while a side stream is current, work.wait() on that stream, a second
gather behind it and the main stream's wait for both.  Prints one JSON line.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    import torch
    import torch.distributed as dist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    from drivers.reddit import synthetic_reddit
    from sgc_amd.distributed import (FeaturePartitionedPropagator, LinePartitionedPropagator,
                                     make_shard)
    from sgc_amd.propagate import csr_of, propagate
    adj, _, features, _, _, _, _ = synthetic_reddit(n)  # on cuda:0
    csr = csr_of(adj)
    X = features
    want = propagate(csr, X, 2)
    rec = {"backend": dist.get_backend(), "world": dist.get_world_size()}
    fp = FeaturePartitionedPropagator(csr, chunks=3)
    fp.force_collectives = True
    got = fp.propagate(X, 2, output="replicated")
    again = fp.propagate(X, 2, output="replicated")
    torch.cuda.synchronize()
    rec["features_replicated_equal"] = bool(torch.equal(got, want) and torch.equal(again, want))
    rp, ci, va = (t.cpu().numpy() for t in (csr.row_ptr, csr.col_idx, csr.val))
    lp = LinePartitionedPropagator(make_shard(rp, ci, va, 0, 1, dev), csr=csr, chunks=3)
    lp.force_collectives = True
    got = lp.propagate(X, 2, output="replicated")
    sh = lp.propagate(X, 2, output="sharded")
    torch.cuda.synchronize()
    rec["lines_replicated_equal"] = bool(torch.equal(got, want))
    rec["lines_sharded_equal"] = bool(torch.equal(sh, want))
    # the product's 1:3:3:1 chunks and the measured-and-not-kept schedules of
    # the replicated last hop (two alternating streams; the hub chunk's hub
    # rows launched early on a third): the same bits
    import sgc_amd.distributed as D
    saved = (D.CHUNK_STREAMS, D.HUB_EARLY)
    ok = True
    try:
        for streams, hub in ((1, False), (2, False), (2, True), (1, True)):
            D.CHUNK_STREAMS, D.HUB_EARLY = streams, hub
            for prop in (FeaturePartitionedPropagator(csr, chunks=4),
                         LinePartitionedPropagator(make_shard(rp, ci, va, 0, 1, dev), csr=csr,
                                                   chunks=4)):
                prop.force_collectives = True
                got = prop.propagate(X, 2, output="replicated")
                torch.cuda.synchronize()
                ok = ok and bool(torch.equal(got, want))
    finally:
        D.CHUNK_STREAMS, D.HUB_EARLY = saved
    rec["schedules_equal"] = ok
    # the replicated last hop through the IPC window (sgc_ipc_get_handle,
    # sgc_signal_flag_i32 / sgc_wait_flags_i32, sgc_pull_blocks_f32) at one
    # rank: X, 2X, 4X, X -- the window's halves alternate, so a stale block
    # would show; power-of-two scaling is exact through every fma
    ipc_ok = {}
    scaled = True
    for name, prop in (("features", FeaturePartitionedPropagator(csr, chunks=4)),
                       ("lines", LinePartitionedPropagator(make_shard(rp, ci, va, 0, 1, dev),
                                                           csr=csr, chunks=4))):
        prop.force_ipc = True
        outs = [prop.propagate(X * s, 2, output="replicated") for s in (1.0, 2.0, 4.0, 1.0)]
        torch.cuda.synchronize()
        ipc_ok[name] = bool(prop._ipc is not None and torch.equal(outs[0], want) and
                            torch.equal(outs[3], want))
        scaled = scaled and torch.equal(outs[1], want * 2.0) and torch.equal(outs[2], want * 4.0)
    rec["ipc_features_equal"] = ipc_ok["features"]
    rec["ipc_lines_equal"] = ipc_ok["lines"]
    rec["ipc_scaled_calls_exact"] = bool(scaled)
    # the tail-stream pattern (LinePartitionedPropagator.propagate): gathers
    # issued from a side stream, waited there, then on the main stream
    full = [torch.zeros((64, 96), device=dev) for _ in range(2)]
    for k in range(2):
        with lp._tail_ctx(dev):
            loc = full[k][:64]
            loc.fill_(float(k + 1))
            work = lp._collective("gather", full[k], loc)
            work.wait()
            full[k].mul_(2.0)  # on the side stream, after the gather
        work.wait()
    torch.cuda.current_stream(dev).wait_stream(lp._tail_stream)
    torch.cuda.synchronize()
    rec["tail_stream_pattern_ok"] = bool(torch.all(full[0] == 2.0) and torch.all(full[1] == 4.0))
    print(json.dumps(rec), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
