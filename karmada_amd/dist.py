"""Multi-GPU sharding of the placement path.

Bindings schedule independently against one snapshot under the default feature
gates (SchedulingOvercommitProtection and WorkloadAffinity off), so the path
shards over bindings with no data-path collective. One process per GPU:

  1. rank 0 packs the snapshot once; the packed bytes are broadcast
     (torch.distributed: RCCL over xGMI on GPUs, gloo on CPU) and every other
     rank imports them (kp_snapshot_import) instead of re-packing;
  2. each rank schedules its contiguous binding range: shard_range (equal counts)
     or shard_range_weighted over per-binding costs (binding_costs, the §8(e)
     cost model C + Rep_b * log2 F_b);
  3. the per-rank CSR results are all-gathered in two phases (gather_csr):
     the counts first, then the CSR arrays padded to the largest rank's sizes,
     so every collective is one fixed-size tensor per rank (RCCL's all_gather).

Steps 1 and 3 are setup/teardown around the timed data path (bench.py reports
weak scaling).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from karmada_amd.engine import Engine, Snapshot


def shard_range(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced [lo, hi) of n bindings for `rank` (equal counts)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def binding_costs(replicas: Sequence[int], n_clusters: int, feasible: Optional[Sequence[int]] = None) -> np.ndarray:
    """Per-binding cost of the path, SURVEY.md §8(e): filter/score/estimate touch every
    cluster (C), the division orders F_b candidates for Rep_b seats (Rep_b * log2 F_b).
    F_b is unknown before filtering; without `feasible` it is bounded by C."""
    rep = np.asarray(replicas, dtype=np.float64)
    f = np.full(rep.shape, float(max(1, n_clusters))) if feasible is None else np.maximum(
        1.0, np.asarray(feasible, dtype=np.float64))
    return float(n_clusters) + np.maximum(rep, 0.0) * np.log2(f + 1.0)


def shard_range_weighted(costs: Sequence[float], world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) whose summed cost is closest to total/world: rank r's range
    starts at the first binding whose cost prefix reaches r/world of the total. Every
    binding lands in exactly one range; ranges may be empty."""
    c = np.asarray(costs, dtype=np.float64)
    n = len(c)
    if n == 0:
        return 0, 0
    pre = np.concatenate(([0.0], np.cumsum(c)))
    total = pre[-1]

    def cut(r):
        if r <= 0:
            return 0
        if r >= world:
            return n
        # first index i with pre[i] >= total * r / world, then the nearer of i-1, i
        t = total * r / world
        i = int(np.searchsorted(pre, t, side="left"))
        if i > 0 and (t - pre[i - 1]) < (pre[i] - t):
            i -= 1
        return min(max(i, 0), n)

    lo, hi = cut(rank), cut(rank + 1)
    return lo, max(lo, hi)


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


@dataclass
class Csr:
    """A batch's results as CSR arrays (the kp_results layout)."""
    status: np.ndarray       # int32 [n]
    err_code: np.ndarray     # int32 [n]
    err_arg: np.ndarray      # int64 [n]
    offsets: np.ndarray      # int64 [n + 1]
    cluster_idx: np.ndarray  # int32 [n_targets] (caller cluster index)
    replicas: np.ndarray     # int32 [n_targets]

    @property
    def n_bindings(self) -> int:
        return len(self.status)

    @property
    def n_targets(self) -> int:
        return len(self.cluster_idx)

    @classmethod
    def from_results(cls, r) -> "Csr":
        """Copies an engine-owned api.kp_results (valid until the next engine call)."""
        n, t = int(r.n_bindings), int(r.n_targets)

        def arr(p, k, dt):
            return np.ctypeslib.as_array(p, shape=(k,)).astype(dt, copy=True) if k else np.zeros(0, dt)
        return cls(arr(r.status, n, np.int32), arr(r.err_code, n, np.int32), arr(r.err_arg, n, np.int64),
                   arr(r.offsets, n + 1, np.int64) if n else np.zeros(1, np.int64),
                   arr(r.cluster_idx, t, np.int32), arr(r.replicas, t, np.int32))

    def slice(self, lo: int, hi: int) -> "Csr":
        """Bindings [lo, hi) as their own CSR (offsets rebased to 0)."""
        a, b = int(self.offsets[lo]), int(self.offsets[hi])
        return Csr(self.status[lo:hi].copy(), self.err_code[lo:hi].copy(), self.err_arg[lo:hi].copy(),
                   self.offsets[lo:hi + 1] - a, self.cluster_idx[a:b].copy(), self.replicas[a:b].copy())

    def to_python(self) -> List[dict]:
        from karmada_amd import api
        return api.results_to_python(self.status, self.err_code, self.err_arg, self.offsets, self.cluster_idx,
                                     self.replicas, self.n_bindings)


def gather_csr(local: Csr) -> Csr:
    """All-gathers every rank's CSR (rank order = binding order of the shards) in two
    phases: (n_bindings, n_targets) per rank, then the per-binding and per-target
    arrays padded to the largest rank's sizes. Fixed-size tensors only, so on GPUs
    each phase is one RCCL all_gather over xGMI. Every rank returns the whole CSR."""
    dev = _device()
    world = dist.get_world_size()
    cnt = torch.tensor([local.n_bindings, local.n_targets], dtype=torch.int64, device=dev)
    cnts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt)
    nb = [int(c[0].item()) for c in cnts]
    nt = [int(c[1].item()) for c in cnts]
    mb, mt = max(1, max(nb)), max(1, max(nt))
    # per-binding block: status, err_code, err_arg, local end offsets (int64 rows)
    pb = torch.zeros((4, mb), dtype=torch.int64, device=dev)
    n = local.n_bindings
    if n:
        rows = np.stack([local.status.astype(np.int64), local.err_code.astype(np.int64), local.err_arg,
                         local.offsets[1:] - local.offsets[0]])
        pb[:, :n] = torch.from_numpy(rows).to(dev)
    pt = torch.zeros((2, mt), dtype=torch.int32, device=dev)
    t = local.n_targets
    if t:
        pt[:, :t] = torch.from_numpy(np.stack([local.cluster_idx, local.replicas])).to(dev)
    gb = [torch.empty_like(pb) for _ in range(world)]
    gt = [torch.empty_like(pt) for _ in range(world)]
    dist.all_gather(gb, pb)
    dist.all_gather(gt, pt)
    status, err, arg, offs, idx, rep = [], [], [], [np.zeros(1, np.int64)], [], []
    base = 0
    for r in range(world):
        b = gb[r][:, :nb[r]].cpu().numpy()
        g = gt[r][:, :nt[r]].cpu().numpy()
        status.append(b[0].astype(np.int32))
        err.append(b[1].astype(np.int32))
        arg.append(b[2])
        offs.append(b[3] + base)
        idx.append(g[0])
        rep.append(g[1])
        base += nt[r]
    cat = np.concatenate
    return Csr(cat(status), cat(err), cat(arg), cat(offs), cat(idx), cat(rep))


def gather_results(local: List[dict], dst: int = 0) -> Optional[List[dict]]:
    """Per-binding result dicts of every rank at `dst` via the CSR all-gather.

    The all-gather leaves the whole batch's CSR on every rank (the fixed-size RCCL
    collective over xGMI is cheaper than a gather plus the padding handshake); only
    `dst` converts it to dicts, the others return None. The result must be CSR-shaped
    (status, err, arg, targets), as kp_schedule_batch's is."""
    t = sum(len(r["targets"]) for r in local)
    offs = np.zeros(len(local) + 1, np.int64)
    idx = np.zeros(t, np.int32)
    rep = np.zeros(t, np.int32)
    k = 0
    for i, r in enumerate(local):
        for c, v in r["targets"]:
            idx[k], rep[k] = c, v
            k += 1
        offs[i + 1] = k
    csr = Csr(np.array([r["status"] for r in local], np.int32), np.array([r["err"] for r in local], np.int32),
              np.array([r["arg"] for r in local], np.int64), offs, idx, rep)
    whole = gather_csr(csr)
    return whole.to_python() if dist.get_rank() == dst else None
