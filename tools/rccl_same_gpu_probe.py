"""Can two RCCL ranks share one GPU on this box?  torch.distributed (nccl backend = RCCL), two
processes both on cuda:0: an all_reduce and a send/recv pair.  Prints one line per rank."""
import os
import sys

import torch
import torch.distributed as dist


def main():
    rank = int(os.environ["RANK"])
    dist.init_process_group("nccl", rank=rank, world_size=int(os.environ["WORLD_SIZE"]),
                            device_id=torch.device("cuda:0"))
    x = torch.full((4,), float(rank + 1), device="cuda:0")
    dist.all_reduce(x)
    y = torch.zeros(4, device="cuda:0")
    if rank == 0:
        dist.send(x * 2, 1)
    else:
        dist.recv(y, 0)
    torch.cuda.synchronize()
    print(f"rank {rank}: all_reduce {x.tolist()} recv {y.tolist()}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
