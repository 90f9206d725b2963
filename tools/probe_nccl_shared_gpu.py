#!/usr/bin/env python3
"""Probe: can two RCCL ("nccl" backend) ranks share one GPU, so the bench's RCCL path could be
rehearsed on a 1-GPU lease?  No: RCCL 2.26 refuses it at communicator setup ("Duplicate GPU
detected : rank 0 and rank 1 both on CUDA device"), so only gloo rehearses N > 1 on one GPU
(DESIGN.md §7)."""
import os, sys, torch, torch.distributed as dist, torch.multiprocessing as mp
def w(rank, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=2, device_id=torch.device("cuda", 0))
    t = torch.ones(4, device="cuda:0") * (rank + 1)
    dist.all_reduce(t)
    print("rank", rank, t.tolist(), flush=True)
    dist.destroy_process_group()
if __name__ == "__main__":
    import socket; s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    mp.spawn(w, args=(port,), nprocs=2, join=True)
