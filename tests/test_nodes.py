"""the member-cluster node paths.

- kp_model_grades: getAllocatableModelings over modeling.AddToResourceSummary
  (cluster_status_controller.go:642-677, modeling.go:75-223). The oracle is pinned
  by pkg/modeling/modeling_test.go (tests/golden/modeling.json: TestGetIndex,
  TestAddToResourceSummary, TestSearchLastLessElement, TestInitSummary*); the
  engine (host build here, libkp.so under -m gpu) is compared with the oracle on
  the same vectors and on seeded node sets (pods, requests, the walk's stop).
- kp_node_max_replicas: nodeResourceEstimator.Estimate (noderesource.go:70-131):
  the assumed-workload deduction, MatchNode (nodeSelector, required node affinity,
  tolerations, the unschedulable taint; filter.go:38-99) and the int32 sum of
  MaxDivided. Pinned by server_test.go:43 (5 cases) and TestMatchNode
  (scheduling_simulator_components_test.go:32), tests/golden/nodes_server.json.
- kp_node_max_component_sets: nodeResourceEstimator.EstimateComponents
  (noderesource.go:146-190), the first-fit set simulation over real nodes. Pinned
  by noderesource_test.go:32 (13 cases). The oracle restates the simulator
  literally (one scan per component per set); the engine's closed-form set
  batching is compared with it on seeded node sets.
"""
import ctypes as C
import json
import os
import random

import pytest

import oracle_lib as O
from karmada_amd import api

GOLDEN = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "modeling.json")))
SERVER = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "nodes_server.json")))
L = O.lib()
L.kpo_model_grades.argtypes = [C.POINTER(api.kp_resource_model), C.c_uint32, C.POINTER(api.kp_node), C.c_uint64,
                               C.POINTER(C.c_int64)]
L.kpo_node_max_replicas.argtypes = [C.POINTER(api.kp_node), C.c_uint64, C.POINTER(api.kp_resource), C.c_uint32,
                                    C.POINTER(api.kp_node_claim), C.POINTER(api.kp_assumed_workload), C.c_uint32,
                                    C.POINTER(C.c_int32)]
L.kpo_node_max_component_sets.argtypes = [C.POINTER(api.kp_node), C.c_uint64, C.POINTER(api.kp_node_component),
                                          C.c_uint32, C.POINTER(api.kp_assumed_workload), C.c_uint32,
                                          C.POINTER(C.c_int32)]


def oracle_grades(models, nodes):
    w = api.World()
    ma, nm = w.models(models)
    na, nn = w.nodes(nodes)
    out = (C.c_int64 * max(1, nm))()
    rc = L.kpo_model_grades(ma, nm, na, nn, out)
    return None if rc else [int(out[i]) for i in range(nm)]


def oracle_node_est(nodes, request, claim=None, assumed=None):
    w = api.World()
    na, nn = w.nodes(nodes)
    ra, nr = w.resources(request)
    c = w.node_claim(claim)
    aa, namd = w.assumed_workloads(assumed)
    out = C.c_int32()
    rc = L.kpo_node_max_replicas(na, nn, ra, nr, C.byref(c) if c is not None else None, aa, namd, C.byref(out))
    assert rc == 0
    return int(out.value)


def oracle_node_sets(nodes, comps, assumed=None):
    w = api.World()
    na, nn = w.nodes(nodes)
    ca, nc = w.node_components(comps)
    aa, namd = w.assumed_workloads(assumed)
    out = C.c_int32()
    assert L.kpo_node_max_component_sets(na, nn, ca, nc, aa, namd, C.byref(out)) == 0
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


def rand_req(r):
    op = r.choice(["In", "NotIn", "Exists", "DoesNotExist", "Gt", "Lt", "Bogus"])
    key = r.choice(["zone", "pool", "arch", "rank", "bad key!"])
    if op in ("In", "NotIn"):
        vals = r.sample(["a", "b", "c", "1", "9"], r.randint(0, 2))
    elif op in ("Gt", "Lt"):
        vals = [r.choice(["0", "3", "-1", "x", "5"])] if r.random() < 0.9 else ["1", "2"]
    else:
        vals = [] if r.random() < 0.9 else ["a"]
    return {"key": key, "operator": op, "values": vals}


def rand_field(r):
    op = r.choice(["In", "NotIn", "In", "Exists"])
    key = r.choice(["metadata.name", "metadata.name", "spec.unschedulable"])
    vals = [r.choice([f"n{r.randint(0, 5)}", "", "x"])] if r.random() < 0.9 else ["n1", "n2"]
    return {"key": key, "operator": op, "values": vals}


def rand_affinity(r):
    terms = []
    for _ in range(r.randint(0, 3)):
        t = {}
        if r.random() < 0.8:
            t["matchExpressions"] = [rand_req(r) for _ in range(r.randint(0, 2))]
        if r.random() < 0.3:
            t["matchFields"] = [rand_field(r) for _ in range(r.randint(1, 2))]
        terms.append(t)
    return {"nodeSelectorTerms": terms}


def rand_claim(r):
    if r.random() < 0.2:
        return None
    c = {"nodeSelector": {k: r.choice(["a", "b"]) for k in ("zone", "pool") if r.random() < 0.4}}
    c["tolerations"] = [{"key": r.choice(["gpu", "spot", "", "node.kubernetes.io/unschedulable"]),
                         "operator": r.choice(["Exists", "Equal", "", "Gt"]), "value": r.choice(["true", "x", ""]),
                         "effect": r.choice(["", "NoSchedule", "NoExecute"])} for _ in range(r.randint(0, 3))]
    if r.random() < 0.5:
        c["nodeAffinity"] = rand_affinity(r)
    return c


def rand_comp(r, small=False):
    q = {"cpu": f"{r.choice([100, 250, 500, 1000, 4000])}m", "memory": f"{r.choice([128, 512, 2048, 8192])}Mi"}
    if r.random() < 0.2:
        q["nvidia.com/gpu"] = "1"
    if r.random() < 0.1:
        q = {}
    c = {"replicas": r.choice([0, 1, 1, 2, 3, 5]) if small else r.choice([0, 1, 2, 4, 7, 20])}
    if r.random() < 0.9:
        c["replicaRequirements"] = {"resourceRequest": q}
        if r.random() < 0.4:
            c["replicaRequirements"]["nodeClaim"] = rand_claim(r)
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
        assumed = [{"components": [rand_comp(r, True) for _ in range(r.randint(0, 2))]}
                   for _ in range(r.randint(0, 2))] if r.random() < 0.5 else None
        assert engine.node_max_replicas(nodes, req, claim, assumed) == oracle_node_est(nodes, req, claim, assumed), \
            (seed, trial)


def check_sets_random(engine, seed, n, trials=6):
    r = random.Random(1000 + seed)
    for trial in range(trials):
        nodes = [rand_node(r, i) for i in range(n)]
        comps = [rand_comp(r) for _ in range(r.randint(1, 4))]
        assumed = [{"components": [rand_comp(r, True) for _ in range(r.randint(0, 2))]}
                   for _ in range(r.randint(0, 2))] if r.random() < 0.4 else None
        want = oracle_node_sets(nodes, comps, assumed)
        assert engine.node_max_component_sets(nodes, comps, assumed) == want, (seed, trial, n)


@pytest.mark.parametrize("seed,n", SEEDS)
def test_nodes_random_cpusim(cpusim_engine, seed, n):
    check_random(cpusim_engine, seed, n)


SET_SEEDS = [(1, 1), (2, 7), (3, 40), (4, 150), (5, 3)]


@pytest.mark.parametrize("seed,n", SET_SEEDS)
def test_node_sets_random_cpusim(cpusim_engine, seed, n):
    check_sets_random(cpusim_engine, seed, n)


def server_case(engine, c):
    if engine is None:
        return oracle_node_est(c["nodes"], c["request"], c.get("claim"))
    return engine.node_max_replicas(c["nodes"], c["request"], c.get("claim"))


def sets_case(engine, c):
    if engine is None:
        return oracle_node_sets(c["nodes"], c["components"], c.get("assumed"))
    return engine.node_max_component_sets(c["nodes"], c["components"], c.get("assumed"))


def check_server_golden(engine):
    for c in SERVER["server"]:
        assert server_case(engine, c) == c["want"], c["name"]
    for c in SERVER["match_node"]:
        assert (server_case(engine, c) > 0) == c["match"], c["name"]
    for c in SERVER["components"]:
        assert sets_case(engine, c) == c["want"], c["name"]


def test_server_golden_oracle():
    check_server_golden(None)


def test_server_golden_cpusim(cpusim_engine):
    check_server_golden(cpusim_engine)


def test_node_affinity_cases(cpusim_engine):
    """Hand-checked node-affinity edges (nodeaffinity.go:39-333): terms are ORed,
    an empty term or one that fails to parse never matches, a selector with no
    usable term matches nothing, matchFields see only metadata.name (and are
    skipped for a nameless node), Gt/Lt parse the node's label value."""
    nodes = [{"name": "n0", "labels": {"rank": "5", "zone": "a"}, "allocatable": {"cpu": "1", "pods": "10"}},
             {"name": "n1", "labels": {"rank": "x", "zone": "b"}, "allocatable": {"cpu": "2", "pods": "10"}},
             {"name": "", "labels": {"zone": "c"}, "allocatable": {"cpu": "4", "pods": "10"}}]
    req = {"cpu": "1"}

    def aff(*terms):
        return {"nodeAffinity": {"nodeSelectorTerms": list(terms)}}

    def me(key, op, *vals):
        return {"matchExpressions": [{"key": key, "operator": op, "values": list(vals)}]}

    def mf(op, *vals, key="metadata.name"):
        return {"matchFields": [{"key": key, "operator": op, "values": list(vals)}]}

    cases = [
        (aff(), 0),                                  # no usable term: nothing matches
        (aff({}), 0),                                # empty term selects nothing
        (aff(me("rank", "Gt", "3")), 1),             # n0 (5 > 3); n1's "x" does not parse
        (aff(me("rank", "Lt", "3")), 0),
        (aff(me("rank", "Gt", "x")), 0),             # parse error: the term never matches
        (aff(me("zone", "In", "a"), me("zone", "In", "c")), 1 + 4),
        (aff(me("zone", "NotIn", "a")), 2 + 4),
        (aff(me("zone", "Bogus")), 0),
        (aff(mf("In", "n1")), 2 + 4),                # the nameless node has no fields: skipped
        (aff(mf("NotIn", "n1")), 1 + 4),
        (aff(mf("In", "n1", "n0")), 0),              # field In needs exactly one value
        (aff(mf("In", "", key="spec.x")), 1 + 2 + 4),  # absent field reads "" (n0, n1); nameless node skips
        (aff(mf("NotIn", "", key="spec.x")), 4),
        ({"nodeSelector": {"zone": "b"}, **aff(me("rank", "Exists"))}, 2),
    ]
    for claim, want in cases:
        assert oracle_node_est(nodes, req, claim) == want, claim
        assert cpusim_engine.node_max_replicas(nodes, req, claim) == want, claim


def test_node_sets_cases(cpusim_engine):
    """Hand-checked first-fit sets: batching across many sets, spanning nodes,
    the pod bound, a zero-replica set, negative replicas (resources returned)."""
    big = [{"name": f"n{i}", "allocatable": {"cpu": "64", "memory": "256Gi", "pods": "110"}} for i in range(50)]
    one = [{"replicas": 1, "replicaRequirements": {"resourceRequest": {"cpu": "250m", "memory": "1Gi"}}}]
    # per node min(64000/250, 256, 110) = 110 pods -> 50 * 110 sets
    assert cpusim_engine.node_max_component_sets(big, one) == 5500 == oracle_node_sets(big, one)
    two = one + [{"replicas": 3, "replicaRequirements": {"resourceRequest": {"cpu": "1", "memory": "4Gi"}}}]
    assert cpusim_engine.node_max_component_sets(big, two) == oracle_node_sets(big, two)
    zero = [{"replicas": 0}]
    assert cpusim_engine.node_max_component_sets(big, zero) == 2147483647 == oracle_node_sets(big, zero)
    neg = [{"replicas": 2, "replicaRequirements": {"resourceRequest": {"cpu": "1"}}},
           {"replicas": -1, "replicaRequirements": {"resourceRequest": {"cpu": "1"}}}]
    small = [{"name": "a", "allocatable": {"cpu": "4", "pods": "10"}}]
    assert cpusim_engine.node_max_component_sets(small, neg) == oracle_node_sets(small, neg)


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
        assert e.node_max_replicas([n1], req, {"nodeAffinity": {}}) == 0 == oracle_node_est([n1], req, {"nodeAffinity": {}})
        with pytest.raises(EngineError):
            e.node_max_replicas([n1], {"cpu": "x"})


@pytest.mark.gpu
def test_nodes_gpu(gpu_engine):
    for case in GOLDEN["cases"]:
        assert engine_grades(gpu_engine, case["models"], case["nodes"]) == (None if case.get("error") else case["counts"])
    for seed, n in SEEDS + [(6, 20000)]:
        check_random(gpu_engine, seed, n)
    check_server_golden(gpu_engine)
    for seed, n in SET_SEEDS + [(6, 300)]:
        check_sets_random(gpu_engine, seed, n, trials=4)
