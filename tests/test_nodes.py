"""the member-cluster node paths.

- kp_model_grades: getAllocatableModelings over modeling.AddToResourceSummary
  (cluster_status_controller.go:642-677, modeling.go:75-223). The oracle is pinned
  by pkg/modeling/modeling_test.go (tests/golden/modeling.json: TestGetIndex,
  TestAddToResourceSummary, TestSearchLastLessElement, TestInitSummary*); the
  engine (host build here, libkp.so under -m gpu) is compared with the oracle on
  the same vectors and on seeded node sets (pods, requests, the walk's stop).
- kp_node_max_replicas: nodeResourceEstimator.Estimate (noderesource.go:70-131):
  MatchNode (nodeSelector, tolerations, the unschedulable taint) and the int32 sum
  of MaxDivided. Parity unpinned by reference vectors (its tests need the
  estimator server's informer cache); the oracle restates it line by line and the
  engine is compared with it on seeded node sets, plus hand-checked cases.
"""
import ctypes as C
import json
import os
import random

import pytest

import oracle_lib as O
from karmada_amd import api

GOLDEN = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "modeling.json")))
L = O.lib()
L.kpo_model_grades.argtypes = [C.POINTER(api.kp_resource_model), C.c_uint32, C.POINTER(api.kp_node), C.c_uint64,
                               C.POINTER(C.c_int64)]
L.kpo_node_max_replicas.argtypes = [C.POINTER(api.kp_node), C.c_uint64, C.POINTER(api.kp_resource), C.c_uint32,
                                    C.POINTER(api.kp_node_claim), C.POINTER(C.c_int32)]


def oracle_grades(models, nodes):
    w = api.World()
    ma, nm = w.models(models)
    na, nn = w.nodes(nodes)
    out = (C.c_int64 * max(1, nm))()
    rc = L.kpo_model_grades(ma, nm, na, nn, out)
    return None if rc else [int(out[i]) for i in range(nm)]


def oracle_node_est(nodes, request, claim=None):
    w = api.World()
    na, nn = w.nodes(nodes)
    ra, nr = w.resources(request)
    c = w.node_claim(claim)
    out = C.c_int32()
    rc = L.kpo_node_max_replicas(na, nn, ra, nr, C.byref(c) if c is not None else None, C.byref(out))
    assert rc == 0
    return int(out.value)


def engine_grades(engine, models, nodes):
    from karmada_amd.engine import EngineError
    try:
        return engine.model_grades(models, nodes)
    except EngineError:
        return None


@pytest.mark.parametrize("case", GOLDEN["cases"], ids=[c["name"] for c in GOLDEN["cases"]])
def test_model_grades_golden_oracle(case):
    got = oracle_grades(case["models"], case["nodes"])
    assert got == (None if case.get("error") else case["counts"])


@pytest.mark.parametrize("case", GOLDEN["cases"], ids=[c["name"] for c in GOLDEN["cases"]])
def test_model_grades_golden_cpusim(cpusim_engine, case):
    assert engine_grades(cpusim_engine, case["models"], case["nodes"]) == (None if case.get("error") else case["counts"])


def rand_models(r):
    k = r.randint(1, 8)
    names = r.sample(["cpu", "memory", "ephemeral-storage", "nvidia.com/gpu"], r.randint(1, 3))
    mins = {n: sorted(r.randint(0, 64) for _ in range(k)) for n in names}
    unit = {"cpu": "", "memory": "Gi", "ephemeral-storage": "Gi", "nvidia.com/gpu": ""}
    return [{"grade": g, "ranges": [{"name": n, "min": f"{mins[n][g]}{unit[n]}", "max": "1000Gi"} for n in names]}
            for g in range(k)]


def rand_node(r, i):
    d = {"name": f"n{i}", "allocatable": {"cpu": f"{r.randint(0, 96000)}m", "memory": f"{r.randint(0, 512)}Gi",
                                          "pods": str(r.randint(0, 120)), "ephemeral-storage": f"{r.randint(0, 80)}Gi"}}
    if r.random() < 0.3:
        d["allocatable"]["nvidia.com/gpu"] = str(r.randint(0, 8))
    if r.random() < 0.7:
        d["pods"] = r.randint(0, 30)
        d["requested"] = {"cpu": f"{r.randint(0, 64000)}m", "memory": f"{r.randint(0, 300)}Gi"}
        if r.random() < 0.3:
            d["requested"]["nvidia.com/gpu"] = str(r.randint(0, 4))
    d["labels"] = {k: r.choice(["a", "b", "c"]) for k in ("zone", "pool", "arch") if r.random() < 0.7}
    if r.random() < 0.3:
        d["taints"] = [{"key": r.choice(["gpu", "spot"]), "value": r.choice(["true", "x"]),
                        "effect": r.choice(["NoSchedule", "NoExecute", "PreferNoSchedule"])}]
    d["unschedulable"] = r.random() < 0.1
    return d


def rand_claim(r):
    if r.random() < 0.2:
        return None
    c = {"nodeSelector": {k: r.choice(["a", "b"]) for k in ("zone", "pool") if r.random() < 0.4}}
    c["tolerations"] = [{"key": r.choice(["gpu", "spot", "", "node.kubernetes.io/unschedulable"]),
                         "operator": r.choice(["Exists", "Equal", "", "Gt"]), "value": r.choice(["true", "x", ""]),
                         "effect": r.choice(["", "NoSchedule", "NoExecute"])} for _ in range(r.randint(0, 3))]
    return c


def rand_request(r):
    q = {"cpu": f"{r.choice([100, 250, 500, 1000, 4000])}m", "memory": f"{r.choice([128, 512, 2048, 8192])}Mi"}
    if r.random() < 0.3:
        q["nvidia.com/gpu"] = "1"
    if r.random() < 0.1:
        q["ephemeral-storage"] = "1Gi"
    return q


SEEDS = [(s, n) for s, n in [(1, 40), (2, 300), (3, 1), (4, 2000), (5, 77)]]


def check_random(engine, seed, n):
    r = random.Random(seed)
    for trial in range(6):
        models = rand_models(r)
        nodes = [rand_node(r, i) for i in range(n)]
        assert engine_grades(engine, models, nodes) == oracle_grades(models, nodes), (seed, trial)
        req, claim = rand_request(r), rand_claim(r)
        assert engine.node_max_replicas(nodes, req, claim) == oracle_node_est(nodes, req, claim), (seed, trial)


@pytest.mark.parametrize("seed,n", SEEDS)
def test_nodes_random_cpusim(cpusim_engine, seed, n):
    check_random(cpusim_engine, seed, n)


def test_node_estimate_cases(cpusim_engine):
    """Hand-checked: available = allocatable - requested (clamped), pods = allocatable
    pods - pods on the node; MaxDivided = min over the request's positive entries."""
    n1 = {"allocatable": {"cpu": "4", "memory": "8Gi", "pods": "110"}, "requested": {"cpu": "1"}, "pods": 100,
          "labels": {"zone": "a"}}
    n2 = {"allocatable": {"cpu": "2", "memory": "1Gi", "pods": "110"}, "labels": {"zone": "b"},
          "taints": [{"key": "gpu", "value": "true", "effect": "NoSchedule"}]}
    req = {"cpu": "500m", "memory": "256Mi"}
    for e in (cpusim_engine,):
        # n1: min(3000/500, 8Gi/256Mi, 110-100) = min(6, 32, 10) = 6; n2 tainted
        assert e.node_max_replicas([n1, n2], req) == 6 == oracle_node_est([n1, n2], req)
        tol = {"tolerations": [{"key": "gpu", "operator": "Exists"}]}
        # n2: min(2000/500, 1Gi/256Mi, 110) = 4
        assert e.node_max_replicas([n1, n2], req, tol) == 10 == oracle_node_est([n1, n2], req, tol)
        sel = {"nodeSelector": {"zone": "b"}, "tolerations": [{"key": "gpu", "operator": "Exists"}]}
        assert e.node_max_replicas([n1, n2], req, sel) == 4 == oracle_node_est([n1, n2], req, sel)
        assert e.node_max_replicas([], req) == 0
        from karmada_amd.engine import EngineError
        with pytest.raises(EngineError):
            e.node_max_replicas([n1], req, {"nodeAffinity": {}})


@pytest.mark.gpu
def test_nodes_gpu(gpu_engine):
    for case in GOLDEN["cases"]:
        assert engine_grades(gpu_engine, case["models"], case["nodes"]) == (None if case.get("error") else case["counts"])
    for seed, n in SEEDS + [(6, 20000)]:
        check_random(gpu_engine, seed, n)
