"""Probe: can two RCCL ranks share one GPU on this pool?

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        scripts/rccl_probe.py

Each rank binds cuda:0, initialises the nccl (RCCL) backend and runs one
all_gather_into_tensor and one all_to_all_single, then checks the result.
Prints one line per rank: ok, or the exception text.
"""
import os
import sys

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    try:
        dist.init_process_group("nccl", device_id=dev)
        x = torch.full((4, 3), float(rank), device=dev)
        y = torch.empty((4 * world, 3), device=dev)
        s = torch.cuda.Stream(dev)
        with torch.cuda.stream(s):
            w = dist.all_gather_into_tensor(y, x, async_op=True)
        w.wait()
        torch.cuda.synchronize()
        want = torch.arange(world, device=dev, dtype=torch.float32).repeat_interleave(4)
        ok_g = bool(torch.equal(y[:, 0], want))
        a = torch.full((world * 2,), float(rank), device=dev)
        b = torch.empty_like(a)
        dist.all_to_all_single(b, a)
        torch.cuda.synchronize()
        ok_a = bool(torch.equal(b, torch.arange(world, device=dev, dtype=torch.float32)
                                .repeat_interleave(2)))
        print(f"rank {rank}: all_gather {'ok' if ok_g else 'WRONG'}, all_to_all "
              f"{'ok' if ok_a else 'WRONG'}", flush=True)
        dist.destroy_process_group()
    except Exception as e:  # report, do not hang
        print(f"rank {rank}: {type(e).__name__}: {e}", flush=True)
        sys.exit(3)


if __name__ == "__main__":
    main()
