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
    from sgc_amd.utils import sgc_precompute
    adj, _, features, _, _, _, _ = synthetic_reddit(n)
    out, secs = sgc_precompute(features, adj, 2)
    out2, _ = sgc_precompute(features, adj, 2)
    rec = {"sha": hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest(),
           "repeat_equal": bool(torch.equal(out, out2)), "seconds": secs,
           "device": str(features.device),
           "world": dist.get_world_size() if dist.is_initialized() else 1,
           "backend": dist.get_backend() if dist.is_initialized() else None}
    rank = int(os.environ.get("RANK", "0"))
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(rec, f)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
