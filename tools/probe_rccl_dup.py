#!/usr/bin/env python3
"""Can RCCL put two ranks of one communicator on the same GPU? (torch "nccl")

Run: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1
     --master-port P tools/probe_rccl_dup.py
Both ranks use cuda:0; prints one line per rank with the all-reduce result or
the error. Used to decide whether multi-rank RCCL tests can run on a 1-GPU box.
"""
import os

import torch
import torch.distributed as dist


def main():
    rank = int(os.environ["RANK"])
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    try:
        dist.init_process_group("nccl", device_id=dev)
        t = torch.full((4,), rank + 1, dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        torch.cuda.synchronize()
        print(f"rank {rank}: ok {t.tolist()}", flush=True)
        dist.destroy_process_group()
    except Exception as e:
        print(f"rank {rank}: error {e!r}"[:400], flush=True)


if __name__ == "__main__":
    main()
