"""One process per GPU: independent problem instances (config C5), one gather of the results at the end.

Nothing is exchanged during a solve: the only collectives are the timing barrier, a MAX
all-reduce of the elapsed time and a gather of {x, stats} to rank 0 (RCCL over xGMI when backend="nccl",
gloo on CPU for the tests).
"""
from __future__ import annotations

import os
from typing import List, Optional

import numpy as np


def env_rank():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))


def init(backend: str):
    import torch.distributed as dist
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend=backend)
    return dist


def max_over_ranks(value: float, device) -> float:
    import torch
    import torch.distributed as dist
    t = torch.tensor([value], dtype=torch.float64, device=device)
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(device):
    import torch
    import torch.distributed as dist
    if dist.is_initialized() and dist.get_world_size() > 1:
        if device.type == "cuda":
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()


def gather_results(x: np.ndarray, stats: np.ndarray, device) -> Optional[List[np.ndarray]]:
    """Gather one fixed-size record [stats..., x...] per rank to rank 0 (the single result collective)."""
    import torch
    import torch.distributed as dist
    rec = torch.from_numpy(np.concatenate([stats.astype(np.float64), x.astype(np.float64)])).to(device)
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return [rec.cpu().numpy()]
    world = dist.get_world_size()
    rank = dist.get_rank()
    out = [torch.empty_like(rec) for _ in range(world)] if rank == 0 else None
    dist.gather(rec, gather_list=out, dst=0)
    if rank != 0:
        return None
    return [o.cpu().numpy() for o in out]
