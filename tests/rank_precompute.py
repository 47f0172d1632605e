"""Helper run under torchrun by tests/test_gpu_multigpu.py (not a test module).

    python -m torch.distributed.run --nproc-per-node N tests/rank_precompute.py OUT_DIR [n]

Each rank builds the same seeded Reddit-shape graph the reddit driver's
--synthetic mode builds (drivers/reddit.py:synthetic_reddit), moves it to
`.cuda()` -- its own GPU, bound by the drop-in under torchrun -- and calls the
unchanged `sgc_precompute(features, adj, 2)` (reference reddit.py:43).  It
writes the SHA-256 of the X_K it got back, the world size and the backend
sgc_precompute chose to OUT_DIR/rank<r>.json.
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out_dir = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    import torch
    import torch.distributed as dist

    from drivers.reddit import synthetic_reddit
    from sgc_amd import multigpu
    from sgc_amd.utils import sgc_precompute
    adj, _, features, _, _, _, _ = synthetic_reddit(n)
    # what the drop-in loaders do once the data is on the GPU (load_reddit_data
    # -> propagate.warmup: code objects, and under torchrun the process group)
    from sgc_amd.propagate import warmup
    warm_s = warmup(features.device)
    outs, secs, props = [], [], []
    for _ in range(3):  # the first call (reddit.py:43 times it), then steady calls
        before = multigpu.PROPAGATIONS[0]
        o, s = sgc_precompute(features, adj, 2)
        props.append(multigpu.PROPAGATIONS[0] - before)
        outs.append(o)
        secs.append(s)
    csr = adj._sgc_amd_csr[1]
    rec = {"sha": hashlib.sha256(outs[0].cpu().numpy().tobytes()).hexdigest(),
           "repeat_equal": all(bool(torch.equal(outs[0], o)) for o in outs[1:]),
           "seconds": secs[0], "call_seconds": secs, "propagations": props,
           "ingest_seconds": getattr(csr, "ingest_seconds", None), "warmup_seconds": warm_s,
           "device": str(features.device),
           "world": dist.get_world_size() if dist.is_initialized() else 1,
           "backend": dist.get_backend() if dist.is_initialized() else None}
    from sgc_amd.distributed import SETUP_SECONDS
    if SETUP_SECONDS:  # SGC_AMD_SETUP_TRACE=1: the set-up stages, host seconds
        rec["setup_seconds"] = {k: round(v, 6) for k, v in SETUP_SECONDS.items()}
    if dist.is_initialized():
        rec["auto"] = multigpu.auto_choice(csr, dist.group.WORLD, features.shape[1], 2)
        props_ = [p for p in csr._plans.values() if hasattr(p, "ipc_unavailable")]
        rec["exchange"] = sorted({"ipc" if getattr(p, "_ipc", None) is not None else "collective"
                                  for p in props_})
    rank = int(os.environ.get("RANK", "0"))
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(rec, f)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
