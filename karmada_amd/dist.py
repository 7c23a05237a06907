"""Multi-GPU sharding of the placement path.

Bindings schedule independently against one snapshot under the default feature
gates, so the path shards over bindings. One process per GPU:

  1. rank 0 packs the snapshot once; the packed bytes are broadcast
     (torch.distributed: RCCL over xGMI on GPUs, gloo on CPU) and every other
     rank imports them (kp_snapshot_import) instead of re-packing;
  2. each rank schedules its contiguous binding range (shard_range);
  3. the per-rank CSR results are gathered to rank 0 (gather_results).

Steps 1 and 3 are setup/teardown around the timed data path, which has no
collective (bench.py reports weak scaling).
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from karmada_amd.engine import Engine, Snapshot


def shard_range(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced [lo, hi) of n bindings for `rank`."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def _device():
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")


def broadcast_snapshot(engine: Engine, snap: Optional[Snapshot], names: List[str], src: int = 0) -> Snapshot:
    """Rank `src` passes its packed snapshot; every rank returns a snapshot on its own engine."""
    dev = _device()
    rank = dist.get_rank()
    if rank == src:
        data = snap.to_bytes()
        n = torch.tensor([len(data)], dtype=torch.int64, device=dev)
    else:
        n = torch.zeros(1, dtype=torch.int64, device=dev)
    dist.broadcast(n, src)
    if rank == src:
        buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    else:
        buf = torch.empty(int(n.item()), dtype=torch.uint8, device=dev)
    dist.broadcast(buf, src)
    if rank == src:
        return snap
    return Snapshot.from_bytes(engine, bytes(buf.cpu().numpy().tobytes()), names)


def gather_results(local: List[dict], dst: int = 0) -> Optional[List[dict]]:
    """Concatenates every rank's per-binding results (rank order) at `dst`."""
    out = [None] * dist.get_world_size() if dist.get_rank() == dst else None
    dist.gather_object(local, out, dst=dst)
    if dist.get_rank() != dst:
        return None
    return [r for part in out for r in part]
