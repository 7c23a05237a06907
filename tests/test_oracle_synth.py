"""The oracle's FAST mode against its FAITHFUL mode on seeded universes.

FAITHFUL runs the reference's literal loops: getMaximumReplicasBasedOnResourceModels'
first-fit over every model node replica by replica (estimator/client/general.go:
111-152 with SchedulingSimulator.SimulateSchedulingFF,
scheduling_simulator_components.go:83-131), the per-binding snapshot deep copy and
the serial assignment. FAST replaces the FF loop by its closed form (every identical
node absorbs exactly its initial MaxDivided) and is the mode the
GPU parity tests compare against, so this pins FAST to FAITHFUL. Cluster and grade
counts are small so the literal FF loop stays tractable.
"""
import ctypes as C

import pytest

from karmada_amd import api, synth
import oracle_lib as O


@pytest.mark.parametrize("config,seed,n_clusters,n_bindings", [
    (3, 51, 24, 160),   # resource-model grades on every cluster
    (6, 52, 30, 200),   # edge workload: NodeClaim, zero/negative grades, summaries, non-workloads
    (2, 53, 20, 200),
    (4, 54, 30, 200),
    (7, 55, 16, 150),
])
def test_fast_matches_faithful_schedule(config, seed, n_clusters, n_bindings):
    u = synth.Universe(config, seed, n_clusters, 0, n_bindings)
    opts = api.options()
    a = O.schedule_c(u.clusters, u.n_clusters, u.bindings, u.n_bindings, opts, O.FAITHFUL, 8)
    b = O.schedule_c(u.clusters, u.n_clusters, u.bindings, u.n_bindings, opts, O.FAST, 8)
    bad = [i for i, (x, y) in enumerate(zip(a, b)) if x != y]
    assert not bad, f"{len(bad)} bindings differ, first {bad[:3]}: {a[bad[0]]} vs {b[bad[0]]}"


@pytest.mark.parametrize("gate", [True, False])
def test_fast_matches_faithful_estimator(gate):
    """GeneralEstimator.maxAvailableReplicas per pair (general.go:66-108), both modes."""
    L = O.lib()
    L.kpo_max_available_replicas.restype = C.c_int32
    u = synth.Universe(6, 56, 40, 0, 120)
    opts = api.options(models_gate=gate)
    model_pairs = 0
    for i in range(u.n_bindings):
        for c in range(u.n_clusters):
            args = (C.byref(u.clusters[c]), C.byref(u.bindings[i]), C.byref(opts))
            x = L.kpo_max_available_replicas(*args, O.FAITHFUL)
            y = L.kpo_max_available_replicas(*args, O.FAST)
            assert x == y, (i, c, x, y)
            model_pairs += u.clusters[c].n_resource_models > 0 and u.bindings[i].has_replica_requirements
    assert model_pairs > 1000
