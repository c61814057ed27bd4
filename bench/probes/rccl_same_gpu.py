"""Can two ranks share one GPU over RCCL? (rehearsal of the world>1 collectives on a 1-GPU box)
torchrun --nproc-per-node 2 bench/probes/rccl_same_gpu.py"""
import os
import torch
import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
x = torch.full((1 << 20,), float(rank + 1), device="cuda")
dist.all_reduce(x)
y = torch.empty(1 << 19, device="cuda")
dist.reduce_scatter_tensor(y, torch.arange(1 << 20, device="cuda", dtype=torch.float32))
z = torch.empty(world * 4, device="cuda", dtype=torch.int64)
dist.all_gather_into_tensor(z, torch.full((4,), rank, device="cuda", dtype=torch.int64))
torch.cuda.synchronize()
print(rank, float(x[0]), float(y[0]), z.tolist(), flush=True)
dist.destroy_process_group()
