"""Probe: can two ranks share one GPU under RCCL (nccl backend)?  Used to
decide whether the open-partition all-to-all can be rehearsed on a 1-GPU box."""
import os, torch, torch.distributed as dist
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
x = torch.arange(4 * world, dtype=torch.int64, device="cuda:0") + 100 * rank
y = torch.empty_like(x)
dist.all_to_all_single(y, x)
torch.cuda.synchronize()
print(rank, y.tolist(), flush=True)
dist.destroy_process_group()
