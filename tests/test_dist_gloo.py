"""Sharded placement over torch.distributed (gloo, world_size 2, CPU).

Covers the multi-GPU path of karmada_amd/dist.py end to end without a GPU:
rank 0 packs the snapshot and broadcasts its bytes, rank 1 imports them, each
rank schedules its cost-balanced binding shard (libkp_cpusim.so: the engine and
kernel bodies on the host), the shards' CSR results are all-gathered in two
phases (counts, then padded arrays), and rank 0 checks them against the oracle
over the whole batch.
"""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_clusters, n_bindings, outdir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), KP_CPUSIM_THREADS="2")
    import torch.distributed as dist
    from karmada_amd import api, synth
    from karmada_amd.dist import (Csr, binding_costs, broadcast_snapshot, gather_csr, gather_results,
                                  shard_range_weighted)
    from karmada_amd.engine import PKG, Batch, Engine, Snapshot

    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = Engine(0, lib_path=os.path.join(PKG, "libkp_cpusim.so"))
    # cost-balanced shards over the whole universe's replicas (§8(e) cost model)
    whole = synth.Universe(6, 31, n_clusters, 0, n_bindings)
    costs = binding_costs([whole.bindings[i].replicas for i in range(n_bindings)], n_clusters)
    lo, hi = shard_range_weighted(costs, world, rank)
    u = synth.Universe(6, 31, n_clusters, lo, hi)
    snap = Snapshot.from_structs(eng, u.clusters, u.n_clusters, u.names, api.options()) if rank == 0 else None
    snap = broadcast_snapshot(eng, snap, u.names)
    b = Batch(snap, structs=u.binding_slice(0, u.n_bindings))
    csr = gather_csr(Csr.from_results(b.schedule_raw()))  # two-phase CSR all-gather
    allres = csr.to_python()
    via_dicts = gather_results(b.schedule())
    if rank == 0:
        import oracle_lib as O
        want = O.schedule_c(whole.clusters, whole.n_clusters, whole.bindings, whole.n_bindings, api.options(),
                            O.FAST, 4)
        bad = [i for i in range(n_bindings) if allres[i] != want[i]]
        bad += [i for i in range(n_bindings) if via_dicts[i] != want[i]]
        with open(os.path.join(outdir, "result.txt"), "w") as f:
            f.write(f"{len(allres)} {len(bad)} {hi - lo}\n")
    else:
        with open(os.path.join(outdir, "rank1.txt"), "w") as f:
            f.write(f"{len(allres)} {hi - lo}\n")
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_schedule_gloo_world2(tmp_path):
    n_clusters, n_bindings = 120, 700
    mp.spawn(_worker, args=(2, _free_port(), n_clusters, n_bindings, str(tmp_path)), nprocs=2, join=True)
    n, bad, n0 = map(int, open(tmp_path / "result.txt").read().split())
    n1, m1 = map(int, open(tmp_path / "rank1.txt").read().split())
    assert n == n_bindings and n1 == n_bindings and bad == 0
    assert n0 + m1 == n_bindings and n0 > 0 and m1 > 0


def test_shard_range_weighted_balances_cost():
    import numpy as np
    from karmada_amd.dist import binding_costs, shard_range_weighted
    rng = np.random.default_rng(5)
    for n, world in ((0, 2), (1, 2), (5, 8), (1000, 2), (1000, 3), (1000, 8), (100000, 8)):
        rep = np.floor(np.exp(rng.random(n) * np.log(1000.0))).astype(int)
        costs = binding_costs(rep, 5000)
        spans = [shard_range_weighted(costs, world, r) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == n
        assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
        if n >= 1000:
            part = [costs[lo:hi].sum() for lo, hi in spans]
            assert max(part) - min(part) <= 2 * costs.max()
    # a heavy tail moves the cut: one binding worth half the batch takes a rank alone
    costs = np.ones(101)
    costs[0] = 100.0
    assert shard_range_weighted(costs, 2, 0) == (0, 1)


def test_shard_range_covers_everything():
    from karmada_amd.dist import shard_range
    for n in (0, 1, 7, 100, 101):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


def test_snapshot_bytes_roundtrip():
    from karmada_amd import api, synth
    from karmada_amd.engine import PKG, Batch, Engine, Snapshot
    eng = Engine(0, lib_path=os.path.join(PKG, "libkp_cpusim.so"))
    u = synth.Universe(6, 32, 90, 0, 400)
    s1 = Snapshot.from_structs(eng, u.clusters, u.n_clusters, u.names, api.options(empty_workload_propagation=True))
    data = s1.to_bytes()
    s2 = Snapshot.from_bytes(eng, data, u.names)
    assert s2.to_bytes() == data
    r1 = Batch(s1, structs=u.binding_slice(0, 400)).schedule()
    r2 = Batch(s2, structs=u.binding_slice(0, 400)).schedule()
    assert r1 == r2
    with pytest.raises(Exception):
        Snapshot.from_bytes(eng, data[: len(data) // 2], u.names)
