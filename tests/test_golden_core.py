"""Reference assignment tests (tests/golden/core.json, transcribed from
pkg/scheduler/core/{generic_scheduler,common,division_algorithm}_test.go)
through the oracle's unit hooks. Results are compared the way each reference
test compares them: Test_DistributionOfReplicas and TestAssignReplicas element
by element in order (reflect.DeepEqual / index-wise asserts), TestSelectClusters
as a set (assert.ElementsMatch), Test_dynamicDivideReplicas as a multiset
(helper.IsScheduleResultEqual).
"""
import ctypes as C
import json
import os

import pytest

import oracle_lib as O
from karmada_amd import api

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CORE = json.load(open(os.path.join(GOLDEN, "core.json")))
L = O.lib()
L.kpo_dynamic_divide.argtypes = [C.POINTER(api.kp_target_cluster), C.c_uint32, C.c_int32, C.c_int32, C.c_int,
                                 C.POINTER(api.kp_binding), C.POINTER(C.c_int32), C.POINTER(api.kp_target_cluster),
                                 C.c_uint32]


def ids(cases):
    return [c["name"] for c in cases]


def assign(case):
    """core.AssignReplicas over the case's ClusterDetailInfo list: [(name, replicas)] or None on error."""
    w = api.World()
    cl = case["clusters"]
    objs = [d["cluster"] or {"name": d["name"]} for d in cl]
    ca, nc = w.clusters(objs)
    cs = (O.kpo_candidate * max(1, len(cl)))(*[
        O.kpo_candidate(w.s(d["name"]), d["score"], d["ovf"], d["avail"], d["alloc"], i) for i, d in enumerate(cl)])
    b = w.binding(case["binding"])
    ec, ea = C.c_int32(), C.c_int64()
    out = (api.kp_target_cluster * 64)()
    k = L.kpo_assign_replicas(cs, len(cl), ca, nc, C.byref(b), 0, C.byref(ec), C.byref(ea), out, 64)
    if k < 0:
        return None
    return [(out[i].name.ptr[:out[i].name.len].decode(), out[i].replicas) for i in range(k)]


@pytest.mark.parametrize("case", CORE["distribution"], ids=ids(CORE["distribution"]))
def test_distribution_of_replicas(case):
    assert assign(case) == [(t["name"], t["replicas"]) for t in case["want"]]


@pytest.mark.parametrize("case", CORE["assign"], ids=ids(CORE["assign"]))
def test_assign_replicas(case):
    got = assign(case)
    if case["wantErr"]:
        assert got is None
    else:
        assert got == [(t["name"], t["replicas"]) for t in case["want"]]


@pytest.mark.parametrize("case", CORE["select"], ids=ids(CORE["select"]))
def test_select_clusters(case):
    w = api.World()
    ca, n = w.clusters(case["clusters"])
    sc = (C.c_int64 * n)(*case["scores"])
    av = (C.c_int32 * n)(*([0] * n))
    b = w.binding(case["binding"])
    out = (C.c_uint32 * 64)()
    k = L.kpo_select_clusters(ca, sc, av, n, C.byref(b), case["binding"].get("replicas", 0), out, 64)
    if case["wantErr"]:
        assert k < 0
    else:
        assert sorted(case["clusters"][out[i]]["name"] for i in range(k)) == case["want"]


@pytest.mark.parametrize("case", CORE["dynamic_divide"], ids=ids(CORE["dynamic_divide"]))
def test_dynamic_divide_replicas(case):
    w = api.World()
    av = case["available"]
    arr, n = w.arr(api.kp_target_cluster, [api.kp_target_cluster(w.s(t["name"]), t["replicas"]) for t in av])
    b = w.binding(case["binding"])
    ec = C.c_int32()
    out = (api.kp_target_cluster * 64)()
    k = L.kpo_dynamic_divide(arr, n, case["availableReplicas"], case["target"], case["strategy"], C.byref(b),
                             C.byref(ec), out, 64)
    if case["wantErr"]:
        assert k < 0
        return
    got = sorted((out[i].name.ptr[:out[i].name.len].decode(), out[i].replicas) for i in range(k))
    assert got == sorted((t["name"], t["replicas"]) for t in case["want"])
