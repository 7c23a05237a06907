"""The multi-GPU engine behind the C-ABI (kp_multi_*, karmada_amd/csrc/multi.cpp):
one process over N devices, the snapshot replicated device to device
(kp_snapshot_replicate), each batch cut into cost-balanced shards scheduled
concurrently and merged into one CSR. SURVEY §8(b) Threading / §8(e); replaces the
reference scheduler's single worker (pkg/scheduler/scheduler.go:327).

CPU: the engine's host build emulates several devices (KP_CPUSIM_DEVICES), so the
orchestration (replicas, shard cuts, the concurrent shards, the merge, updates) is
checked against the oracle on every CPU run. GPU: the same path on the box's one
MI355X (n = 1), and a replica made on the same device by the peer-copy route.
"""
import ctypes as C
import math
import os

import pytest

from karmada_amd import api, synth
from karmada_amd.engine import PKG, Batch, Engine, MultiBatch, MultiEngine, Snapshot, load_library
import oracle_lib as O

CPUSIM = os.path.join(PKG, "libkp_cpusim.so")


def oracle(u, opts):
    return O.schedule_c(u.clusters, u.n_clusters, u.bindings, u.n_bindings, opts, O.FAST, 8)


def compare(got, want, label):
    assert len(got) == len(want)
    bad = [i for i, (g, w) in enumerate(zip(got, want)) if g != w]
    if bad:
        lines = [f"{label}: {len(bad)}/{len(want)} differ"]
        for i in bad[:4]:
            lines += [f"  {i}: got={got[i]}", f"  {i}: ref={want[i]}"]
        pytest.fail("\n".join(lines))


def multi_schedule(lib, devices, u, opts):
    m = MultiEngine(devices, lib_path=lib)
    s = m.snapshot(u.clusters, u.n_clusters, opts)
    b = MultiBatch(s, u.binding_slice(0, u.n_bindings))
    cuts = b.shards()
    out = b.schedule()
    b.close()
    s.close()
    m.close()
    return out, cuts


@pytest.mark.parametrize("devices", [[0, 1], [3, 1, 2]], ids=["2dev", "3dev"])
@pytest.mark.parametrize("config,seed,n_clusters,n_bindings", [
    (3, 3, 200, 300), (4, 4, 400, 500), (6, 6, 120, 900), (7, 17, 300, 400), (8, 4, 64, 300),
])
def test_multi_cpusim_parity(devices, config, seed, n_clusters, n_bindings):
    os.environ.setdefault("KP_CPUSIM_THREADS", "4")
    u = synth.Universe(config, seed, n_clusters, 0, n_bindings)
    opts = api.options()
    got, cuts = multi_schedule(CPUSIM, devices, u, opts)
    assert cuts[0] == 0 and cuts[-1] == n_bindings and cuts == sorted(cuts) and len(cuts) == len(devices) + 1
    compare(got, oracle(u, opts), f"multi {devices} config {config}")


def test_shard_cuts_cost_balanced():
    """Equal prefix sums of C + Replicas*log2 C (SURVEY §8(e) cost model)."""
    L = load_library(CPUSIM)
    w = api.World()
    reps = [1] * 50 + [1000] * 10 + [1] * 40
    ba, n = w.bindings([{"replicas": r} for r in reps])
    C_ = 100
    out = (C.c_uint64 * 5)()
    assert L.kp_multi_shard_cuts(ba, n, C_, 4, out) == 0
    cuts = list(out)
    assert cuts[0] == 0 and cuts[4] == n
    cost = [C_ + r * math.log2(C_) for r in reps]
    tot = sum(cost)
    for d in range(1, 4):
        # the d-th cut is the first index whose prefix reaches d/4 of the total
        pre = sum(cost[:cuts[d]])
        assert pre >= tot * d / 4 - 1e-6
        assert sum(cost[:cuts[d] - 1]) < tot * d / 4
    # an empty batch and more shards than bindings
    assert L.kp_multi_shard_cuts(ba, 0, C_, 3, out) == 0 and list(out)[:4] == [0, 0, 0, 0]
    ba2, n2 = w.bindings([{"replicas": 1}, {"replicas": 1}])
    assert L.kp_multi_shard_cuts(ba2, n2, C_, 4, out) == 0
    assert list(out) == sorted(out) and out[4] == 2


def test_multi_cpusim_update_and_reuse():
    """kp_multi_snapshot_update reaches every replica: a batch scheduled after an
    update matches the oracle on the updated clusters; the batch is re-scheduled
    (its merged result buffers reused) with identical results."""
    u = synth.Universe(6, 6, 120, 0, 600)
    u2 = synth.Universe(6, 66, 120, 0, 1)  # other seed: other cluster contents, same names
    opts = api.options()
    m = MultiEngine([0, 1], lib_path=CPUSIM)
    s = m.snapshot(u.clusters, u.n_clusters, opts)
    grew = s.update_structs(u2.clusters, u2.n_clusters)
    b = MultiBatch(s, u.binding_slice(0, u.n_bindings))
    if grew:  # batches must be packed after a growing update anyway
        pass
    first = b.schedule()
    again = b.schedule()
    assert first == again
    want = O.schedule_c(u2.clusters, u2.n_clusters, u.bindings, u.n_bindings, opts, O.FAST, 8)
    compare(first, want, "multi after update")
    b.close()
    s.close()
    m.close()


def test_replicate_cpusim():
    """kp_snapshot_replicate: a replica on another (emulated) device schedules as its source."""
    u = synth.Universe(4, 4, 300, 0, 400)
    opts = api.options()
    e0, e1 = Engine(0, lib_path=CPUSIM), Engine(1, lib_path=CPUSIM)
    s0 = Snapshot.from_structs(e0, u.clusters, u.n_clusters, u.names, opts)
    h = C.c_void_p()
    e1._check(e1.L.kp_snapshot_replicate(e1.h, s0.h, C.byref(h)), "kp_snapshot_replicate")
    s1 = Snapshot.__new__(Snapshot)
    s1.engine, s1.names, s1.opts, s1.h = e1, u.names, opts, h
    b = Batch(s1, structs=u.binding_slice(0, u.n_bindings))
    compare(b.schedule(), oracle(u, opts), "replica")
    b.close()
    s1.close()
    s0.close()
    e1.close()
    e0.close()


def test_multi_failed_update_invalidates():
    """A kp_multi_snapshot_update that fails on any device leaves the replicas possibly
    different: the multi snapshot refuses batches and schedules (KP_ESTATE)
    until it is rebuilt; a batch created before the failure is refused too."""
    from karmada_amd.engine import EngineError
    u = synth.Universe(6, 6, 60, 0, 50)
    opts = api.options()
    m = MultiEngine([0, 1], lib_path=CPUSIM)
    s = m.snapshot(u.clusters, u.n_clusters, opts)
    b = MultiBatch(s, u.binding_slice(0, u.n_bindings))
    assert len(b.schedule()) == 50
    w = api.World()
    ca, n = w.clusters([{"name": "no-such-cluster"}])
    with pytest.raises(EngineError, match="rc=-1"):
        s.update_structs(ca, n)
    with pytest.raises(EngineError, match="rc=-5"):
        b.schedule()
    with pytest.raises(EngineError, match="rc=-5"):
        MultiBatch(s, u.binding_slice(0, u.n_bindings))
    with pytest.raises(EngineError, match="rc=-5"):
        s.update_structs(u.clusters, u.n_clusters)
    b.close()
    s.close()
    s = m.snapshot(u.clusters, u.n_clusters, opts)  # rebuilt: usable again
    b = MultiBatch(s, u.binding_slice(0, u.n_bindings))
    compare(b.schedule(), oracle(u, opts), "multi after rebuild")
    b.close()
    s.close()
    m.close()


def test_multi_rejects_duplicate_devices():
    L = load_library(CPUSIM)
    devs = (C.c_int * 2)(0, 0)
    h = C.c_void_p()
    assert L.kp_multi_create(devs, 2, C.byref(h)) == -1


@pytest.mark.gpu
@pytest.mark.parametrize("config,seed,n_clusters,n_bindings", [(3, 3, 5000, 2000), (4, 4, 5000, 2000),
                                                               (6, 6, 300, 3000)])
def test_multi_gpu_one_device(config, seed, n_clusters, n_bindings):
    """kp_multi over the box's one MI355X: the same merged CSR as the oracle."""
    u = synth.Universe(config, seed, n_clusters, 0, n_bindings)
    opts = api.options()
    got, cuts = multi_schedule(os.path.join(PKG, "libkp.so"), [0], u, opts)
    assert cuts == [0, n_bindings]
    compare(got, oracle(u, opts), f"multi gpu config {config}")


@pytest.mark.gpu
def test_replicate_gpu_same_device():
    """kp_snapshot_replicate on the GPU (device-to-device copy of the packed image,
    views rebased): the replica schedules exactly as the oracle says."""
    u = synth.Universe(3, 3, 5000, 0, 1000)
    opts = api.options()
    e = Engine(0)
    s0 = Snapshot.from_structs(e, u.clusters, u.n_clusters, u.names, opts)
    h = C.c_void_p()
    e._check(e.L.kp_snapshot_replicate(e.h, s0.h, C.byref(h)), "kp_snapshot_replicate")
    s0.close()  # the replica owns its own copy
    s1 = Snapshot.__new__(Snapshot)
    s1.engine, s1.names, s1.opts, s1.h = e, u.names, opts, h
    b = Batch(s1, structs=u.binding_slice(0, u.n_bindings))
    compare(b.schedule(), oracle(u, opts), "gpu replica")
    b.close()
    s1.close()
    e.close()
