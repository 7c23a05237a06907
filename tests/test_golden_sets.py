"""MaxAvailableComponentSets (estimator/client/general.go:154-292), §8(f)3.

Golden vectors (tests/golden/sets.json, transcribed by make_golden_r2.py):
  models   general_test.go TestGetMaximumSetsBasedOnResourceModels
  general  general_test.go TestGetMaxAvailableComponentSetsGeneral
  ff       scheduling_simulator_components_test.go TestSchedulingSimulator_SimulateSchedulingFF
checked on the oracle in both modes (FAITHFUL: the literal first-fit over every
node; FAST: the run form the device restates), then the engine
(kp_max_available_component_sets; host build here, libkp.so under -m gpu)
against the oracle on the reference's clusters and on seeded universes.
"""
import ctypes as C
import json
import os
import random

import pytest

from karmada_amd import api, synth
from karmada_amd.engine import EngineError, GenericScheduler, Snapshot
import oracle_lib as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SETS = json.load(open(os.path.join(GOLDEN, "sets.json")))
L = O.lib()
for fn in ("kpo_max_sets_models", "kpo_simulate_sets", "kpo_max_available_component_sets"):
    getattr(L, fn).restype = C.c_int32
L.kpo_max_sets_models.argtypes = [C.POINTER(api.kp_cluster), C.POINTER(api.kp_component), C.c_uint32, C.c_int32,
                                  C.c_int]
L.kpo_simulate_sets.argtypes = [C.POINTER(api.kp_cluster), C.c_uint32, C.POINTER(api.kp_component), C.c_uint32,
                                C.c_int32, C.c_int]
L.kpo_max_available_component_sets.argtypes = [C.POINTER(api.kp_cluster), C.POINTER(api.kp_component), C.c_uint32,
                                               C.POINTER(api.kp_options), C.c_int]
MODES = [O.FAITHFUL, O.FAST]


def ids(cases):
    return [c["name"] for c in cases]


def oracle_sets(w, cluster, comps, opts, mode):
    ca, n = w.components(comps)
    return L.kpo_max_available_component_sets(C.byref(cluster), ca, n, C.byref(opts), mode)


@pytest.mark.parametrize("mode", MODES, ids=["faithful", "fast"])
@pytest.mark.parametrize("case", SETS["models"], ids=ids(SETS["models"]))
def test_models_oracle(case, mode):
    w = api.World()
    c = w.cluster(case["cluster"])
    ca, n = w.components(case["components"])
    got = L.kpo_max_sets_models(C.byref(c), ca, n, case["upperBound"], mode)
    assert got == case["expectedSets"]


@pytest.mark.parametrize("mode", MODES, ids=["faithful", "fast"])
@pytest.mark.parametrize("case", SETS["general"], ids=ids(SETS["general"]))
def test_general_oracle(case, mode):
    w = api.World()
    assert oracle_sets(w, w.cluster(case["cluster"]), case["components"], api.options(), mode) == case["expected"]


@pytest.mark.parametrize("mode", MODES, ids=["faithful", "fast"])
@pytest.mark.parametrize("case", SETS["ff"], ids=ids(SETS["ff"]))
def test_ff_simulator_oracle(case, mode):
    w = api.World()
    nodes = [{"name": nd["name"], "resourceSummary": {"allocatable": nd["allocatable"]}} for nd in case["nodes"]]
    na, nn = w.arr(api.kp_cluster, [w.cluster(nd) for nd in nodes])
    ca, n = w.components(case["components"])
    assert L.kpo_simulate_sets(na, nn, ca, n, case["upperBound"], mode) == case["expectedSets"]


def random_components(rng, k):
    cpus = ["100m", "250m", "500m", "1", "2", "3", "4"]
    mems = ["128Mi", "512Mi", "1Gi", "2Gi", "4Gi", "10Gi", "1000000000"]
    out = []
    for i in range(k):
        rr = {"cpu": rng.choice(cpus), "memory": rng.choice(mems)}
        if rng.random() < 0.2:
            rr["nvidia.com/gpu"] = "1"
        c = {"name": "c%d" % i, "replicas": rng.choice([0, 1, 1, 2, 3, 5, 8])}
        if rng.random() < 0.9:
            c["replicaRequirements"] = {"resourceRequest": rr}
        out.append(c)
    return out


def test_fast_matches_faithful_on_synth():
    """Random multi-template sets on seeded model-grade clusters: the run form equals the
    literal first fit (small grade counts keep FAITHFUL tractable)."""
    rng = random.Random(7)
    u = synth.Universe(3, 71, 40, 0, 0)
    opts = api.options()
    w = api.World()
    checked = 0
    for t in range(60):
        comps = random_components(rng, rng.randint(1, 4))
        for c in range(0, u.n_clusters, 3):
            a = oracle_sets(w, u.clusters[c], comps, opts, O.FAITHFUL)
            b = oracle_sets(w, u.clusters[c], comps, opts, O.FAST)
            assert a == b, (t, c, comps, a, b)
            checked += a > 0
    assert checked > 50


def engine_sets(engine, clusters_dicts, comps, opts):
    g = GenericScheduler(engine, clusters_dicts, opts)
    return g.max_available_component_sets(comps, [c["name"] for c in clusters_dicts])


def named(case_cluster, i):
    c = dict(case_cluster)
    c["name"] = "m%d" % i
    return c


def check_engine(engine):
    opts = api.options(multi_templates=True)
    # the reference's clusters: every general case against its own cluster
    for i, case in enumerate(SETS["general"] + SETS["models"]):
        cl = [named(case["cluster"], i)]
        got = engine_sets(engine, cl, case["components"], opts)
        w = api.World()
        want = oracle_sets(w, w.cluster(cl[0]), case["components"], opts, O.FAST)
        assert got == [want], (case["name"], got, want)
    # seeded universes (configs with and without resource models)
    rng = random.Random(11)
    for cfg, seed, C_ in ((3, 72, 120), (6, 73, 150), (2, 74, 60)):
        u = synth.Universe(cfg, seed, C_, 0, 0)
        snap = Snapshot.from_structs(engine, u.clusters, u.n_clusters, u.names, opts)
        g = GenericScheduler.__new__(GenericScheduler)
        g.snapshot = snap
        for t in range(12):
            comps = random_components(rng, rng.randint(1, 5))
            got = g.max_available_component_sets(comps, u.names)
            w = api.World()
            want = [oracle_sets(w, u.clusters[c], comps, opts, O.FAST) for c in range(u.n_clusters)]
            bad = [(c, got[c], want[c]) for c in range(u.n_clusters) if got[c] != want[c]]
            assert not bad, (cfg, t, comps, bad[:5])
        snap.close()


def test_engine_cpusim(cpusim_engine):
    check_engine(cpusim_engine)


def test_gate_off_is_enotsup(cpusim_engine):
    g = GenericScheduler(cpusim_engine, [SETS["general"][3]["cluster"] | {"name": "m"}], api.options())
    with pytest.raises(EngineError):
        g.max_available_component_sets(SETS["general"][3]["components"], ["m"])


@pytest.mark.gpu
def test_engine_gpu(gpu_engine):
    check_engine(gpu_engine)
