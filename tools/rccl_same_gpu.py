"""Can two RCCL ranks share one GPU on this box?  Two processes, backend nccl, both on cuda:0:
all_reduce, all_gather_into_tensor and all_to_all_single with splits on device tensors.
Prints one line per rank; the launcher (torch.distributed.run) sets RANK / WORLD_SIZE."""
import os
import torch
import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
t = torch.full((4,), rank + 1, device="cuda", dtype=torch.int64)
dist.all_reduce(t)
g = torch.empty(4 * world, device="cuda", dtype=torch.int64)
dist.all_gather_into_tensor(g, torch.full((4,), rank, device="cuda", dtype=torch.int64))
send = torch.arange(3, device="cuda", dtype=torch.int64) + 10 * rank
out = torch.empty(3, device="cuda", dtype=torch.int64)
dist.all_to_all_single(out, send, output_split_sizes=[2, 1] if rank == 0 else [1, 2],
                       input_split_sizes=[2, 1] if rank == 0 else [1, 2])
torch.cuda.synchronize()
print(f"rank {rank}: all_reduce {t.tolist()} all_gather {g.tolist()} all_to_all {out.tolist()}", flush=True)
dist.destroy_process_group()
