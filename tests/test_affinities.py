"""kp_schedule_affinities: Scheduler.scheduleResourceBindingWithClusterAffinities
(pkg/scheduler/scheduler.go:618-684) batched, every term retry of a round in one device batch.

- The five cases of the reference's TestScheduleResourceBindingWithClusterAffinities
  (scheduler_test.go:537-808) are restated with real clusters in place of its mock algorithm:
  a term "fails" because its ClusterNames name a cluster absent from the snapshot (FitError).
- Seeded edge-config universes (multi-term affinities with overflow tiers, observed names that
  match, miss or are empty, reschedule triggers) are compared with the oracle's retry driver
  (oracle/oracle.cpp ScheduleWithAffinities): results, chosen term index and attempt count.
The CPU tests run the engine's own code through libkp_cpusim.so; the gpu-marked ones run libkp.so.
"""
import os

import pytest

from karmada_amd import api, synth
from karmada_amd.engine import Engine, GenericScheduler, PKG, Snapshot
import oracle_lib as O

CPUSIM = os.path.join(PKG, "libkp_cpusim.so")
DEPLOY = [{"groupVersion": "apps/v1", "resources": [{"kind": "Deployment"}]}]


def cluster(name):
    return {"name": name, "apiEnablements": DEPLOY}


def terms():
    return [{"affinityName": "affinity1", "clusterNames": ["cluster1"]},
            {"affinityName": "affinity2", "clusterNames": ["cluster2"]}]


# (name, cluster names in the snapshot, binding extras, expected targets, affinity name, attempts, status)
REF_CASES = [
    ("successful scheduling with first affinity", ["cluster1", "cluster2"], {},
     [("cluster1", 1)], "affinity1", 1, api.STATUS_OK),
    ("explicit rescheduling restarts from first affinity", ["cluster1", "cluster2"],
     {"rescheduleTriggeredAt": 2_000_000_000, "lastScheduledTime": 1_000_000_000,
      "schedulerObservedAffinityName": "affinity2"},
     [("cluster1", 1)], "affinity1", 1, api.STATUS_OK),
    ("without explicit rescheduling resumes from observed affinity", ["cluster1", "cluster2"],
     {"schedulerObservedAffinityName": "affinity2"},
     [("cluster2", 1)], "affinity2", 1, api.STATUS_OK),
    ("successful scheduling with second affinity", ["cluster2", "cluster3"], {},
     [("cluster2", 1)], "affinity2", 2, api.STATUS_OK),
    ("all affinities fail", ["cluster3"], {},
     [], None, 2, api.STATUS_FIT_ERROR),
]


def ref_binding(extra):
    b = {"name": "test-binding", "uid": "u-1", "replicas": 1, "placement": {"clusterAffinities": terms()}}
    b.update(extra)
    return b


def run_ref_cases(engine):
    for name, cnames, extra, targets, aff, attempts, status in REF_CASES:
        gs = GenericScheduler(engine, [cluster(c) for c in cnames])
        b = ref_binding(extra)
        w = api.World()
        structs = w.bindings([b])
        res, idx, att, rounds = gs.schedule_affinities_raw(structs)
        sr = gs.schedule_with_affinities([b])[0]
        assert sr.status == status, name
        assert sorted((t.name, t.replicas) for t in sr.suggested_clusters) == targets, name
        assert sr.observed_affinity_name == aff, name
        assert att[0] == attempts and rounds == attempts, name
        # the oracle's retry driver agrees
        wc = api.World()
        ca, nc = wc.clusters([cluster(c) for c in cnames])
        want, widx, watt = O.schedule_affinities_c(ca, nc, structs[0], structs[1], api.options())
        assert (res, idx, att) == (want, widx, watt), name
        gs.snapshot.close()


def run_universe(engine, config, seed, n_clusters, n_bindings):
    u = synth.Universe(config, seed, n_clusters, 0, n_bindings)
    opts = api.options()
    snap = Snapshot.from_structs(engine, u.clusters, u.n_clusters, u.names, opts)
    gs = GenericScheduler.__new__(GenericScheduler)
    gs.snapshot = snap
    ba, n = u.binding_slice(0, n_bindings)
    got = gs.schedule_affinities_raw((ba, n))
    want = O.schedule_affinities_c(u.clusters, u.n_clusters, ba, n, opts, O.FAST, 8)
    snap.close()
    res, idx, att, rounds = got
    bad = [i for i in range(n) if (res[i], idx[i], att[i]) != (want[0][i], want[1][i], want[2][i])]
    assert not bad, [(i, res[i], idx[i], att[i], want[0][i], want[1][i], want[2][i]) for i in bad[:3]]
    assert rounds == max(att)
    return idx, att


@pytest.fixture(scope="module")
def simengine():
    os.environ.setdefault("KP_CPUSIM_THREADS", "8")
    e = Engine(0, lib_path=CPUSIM)
    yield e
    e.close()


def test_reference_cases_cpusim(simengine):
    run_ref_cases(simengine)


@pytest.mark.parametrize("seed,n_clusters,n_bindings", [(6, 120, 1500), (11, 40, 1500), (12, 257, 600)])
def test_universe_cpusim(simengine, seed, n_clusters, n_bindings):
    idx, att = run_universe(simengine, 6, seed, n_clusters, n_bindings)
    assert max(att) >= 2  # some bindings retried a later term
    assert any(a >= 1 for a in idx)


def test_no_affinities_is_one_round(simengine):
    u = synth.Universe(3, 3, 100, 0, 200)
    idx, att = run_universe(simengine, 3, 3, 100, 200)
    assert set(att) == {1} and set(idx) == {-1}


@pytest.fixture(scope="module")
def gpuengine():
    e = Engine(0)
    yield e
    e.close()


@pytest.mark.gpu
def test_reference_cases_gpu(gpuengine):
    run_ref_cases(gpuengine)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n_clusters,n_bindings", [(6, 120, 1500), (11, 40, 1500), (12, 257, 600),
                                                        (13, 5000, 4000)])
def test_universe_gpu(gpuengine, seed, n_clusters, n_bindings):
    idx, att = run_universe(gpuengine, 6, seed, n_clusters, n_bindings)
    assert max(att) >= 2
