"""Host-time breakdown of one public sgc_precompute call at Pubmed shape.

    python scripts/host_breakdown.py [--shape pubmed] [--reps 500]

Medians (us) of each piece of the call's host path, timed on its own:
the whole synchronised call, torch.cuda.synchronize() when idle, csr_of, the
multi-GPU checks (process_group, devices_from_env), check_propagation_inputs,
the result's allocation, propagate()'s enqueue (prepared loop), the
recorded launch list replayed bare (one sgc_launch_list_run call), the GPU
time of the hops (events), and each enqueue followed by a device or stream
synchronise.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sgc_amd import _lib, graphs, multigpu  # noqa: E402
from sgc_amd.propagate import check_propagation_inputs, csr_of, propagate  # noqa: E402
from sgc_amd.utils import sgc_precompute  # noqa: E402


def med(f, reps):
    for _ in range(10):
        f()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter_ns()
        f()
        ts.append(time.perf_counter_ns() - t0)
    return float(np.median(ts)) / 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="pubmed")
    ap.add_argument("--reps", type=int, default=500)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    spec = graphs.SHAPES[a.shape]
    S = graphs.synthetic_graph(a.shape, seed=0)
    X = torch.from_numpy(graphs.synthetic_features(a.shape, S.n, spec["features"], seed=1)).to(dev)
    r, c, v = S.coo()
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.stack([r, c])), torch.from_numpy(v),
                                  (S.n, S.n)).to(dev)
    K = spec["hops"]
    sgc_precompute(X, adj, K)
    csr = csr_of(adj)
    torch.cuda.synchronize()
    rec = {"shape": a.shape, "K": K}
    rec["call_us"] = med(lambda: sgc_precompute(X, adj, K), a.reps)
    rec["sync_idle_us"] = med(torch.cuda.synchronize, a.reps)
    rec["sync_dev_arg_idle_us"] = med(lambda: torch.cuda.synchronize(dev), a.reps)
    rec["current_device_us"] = med(torch.cuda.current_device, a.reps)
    rec["stream_handle_us"] = med(lambda: _lib.stream_handle(dev), a.reps)
    rec["capturing_us"] = med(torch.cuda.is_current_stream_capturing, a.reps)
    rec["csr_of_us"] = med(lambda: csr_of(adj), a.reps)
    rec["process_group_us"] = med(lambda: multigpu.process_group(dev), a.reps)
    rec["devices_from_env_us"] = med(lambda: multigpu.devices_from_env(0), a.reps)
    rec["check_inputs_us"] = med(lambda: check_propagation_inputs(csr, X), a.reps)
    rec["alloc_out_us"] = med(lambda: torch.empty(X.shape, device=dev), a.reps)
    out = torch.empty_like(X)
    propagate(csr, X, K, out=out)

    def enq():
        propagate(csr, X, K, out=out)
    rec["propagate_enqueue_us"] = med(enq, min(a.reps, 200))
    torch.cuda.synchronize()
    rec["device_ctx_us"] = med(lambda: torch.cuda.device(dev).__enter__(), a.reps)
    ev = []
    for _ in range(50):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        propagate(csr, X, K, out=out)
        e.record()
        ev.append((s, e))
    torch.cuda.synchronize()
    rec["gpu_events_us"] = float(np.median([s.elapsed_time(e) for s, e in ev])) * 1e3
    # the synchronised pieces: enqueue + wait, with the device-wide and the
    # stream's synchronise, and the prepared launches replayed bare
    cs = torch.cuda.current_stream(dev)
    rec["propagate_devsync_us"] = med(lambda: (propagate(csr, X, K, out=out),
                                               torch.cuda.synchronize()), a.reps)
    rec["propagate_streamsync_us"] = med(lambda: (propagate(csr, X, K, out=out),
                                                  cs.synchronize()), a.reps)
    prep = [v for k, v in csr._plans.items() if isinstance(k, tuple) and k[:1] == ("list",)]
    handle = prep[-1][1].handle
    lib = _lib.load()
    xp, op, sh = X.data_ptr(), out.data_ptr(), _lib.stream_handle(dev)

    def bare():  # the recorded launch list alone (one ctypes call)
        lib.sgc_launch_list_run(handle, xp, op, sh)
    rec["bare_enqueue_us"] = med(bare, min(a.reps, 200))
    torch.cuda.synchronize()
    rec["bare_devsync_us"] = med(lambda: (bare(), torch.cuda.synchronize()), a.reps)
    def spin():
        ev = torch.cuda.Event()
        ev.record()
        while not ev.query():
            pass
    rec["bare_eventspin_us"] = med(lambda: (bare(), spin()), a.reps)
    rec["propagate_eventspin_us"] = med(lambda: (propagate(csr, X, K, out=out), spin()), a.reps)
    rec["trivial_ctypes_call_us"] = med(lambda: lib.sgc_get_tuning(b"slice_floats"), a.reps)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
