"""Pins the CPU oracle against the reference's own table-driven tests.

Every fixture under tests/golden/ is a hand transcription of a Go test table
(file:line in the fixture's "source"); the expected values are the reference's.
CPU-only (no GPU marker).
"""
import ctypes as C
import json
import os

import pytest

import oracle_lib as O
from karmada_amd import api

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def ids(cases):
    return [c["name"] for c in cases]


def multiset_eq(got, want):
    """helper.IsScheduleResultEqual (test/helper/scheduler.go:26-40)."""
    if len(got) != len(want):
        return False
    return all(any(g[0] == w[0] and g[1] == w[1] for w in want) for g in got)


# --------------------------------------------------------------------------- webster
WEB = load("webster.json")


@pytest.mark.parametrize("case", WEB["cases"], ids=ids(WEB["cases"]))
def test_webster(case):
    L = O.lib()
    w = api.World()
    vn = list(case["votes"].keys())
    names, n = w.arr(api.kp_str, [w.s(x) for x in vn])
    votes = (C.c_int64 * max(1, n))(*[case["votes"][x] for x in vn])
    inn = list(case["init"].keys())
    inames, ni = w.arr(api.kp_str, [w.s(x) for x in inn])
    iseats = (C.c_int32 * max(1, ni))(*[case["init"][x] for x in inn])
    tie = {None: 0, "name_asc": 1, "name_desc": 2}[case["tie"]]
    out = (C.c_int32 * 64)()
    k = L.kpo_allocate_webster(case["newSeats"], names, votes, n, inames, iseats, ni, tie, api.kp_str(None, 0), out, 64)
    allnames = sorted(set(vn) | set(inn))
    assert k == len(allnames)
    got = {allnames[i]: out[i] for i in range(k)}
    assert got == case["expected"]


# --------------------------------------------------------------------------- dispenser
DISP = load("dispenser.json")


@pytest.mark.parametrize("case", DISP["cases"], ids=ids(DISP["cases"]))
def test_dispenser(case):
    L = O.lib()
    w = api.World()
    tcs, n = w.arr(api.kp_target_cluster, [api.kp_target_cluster(w.s(a), b) for a, b in case["weights"]])
    init, ni = w.arr(api.kp_target_cluster, [api.kp_target_cluster(w.s(a), b) for a, b in case["init"]])
    out = (api.kp_target_cluster * 64)()
    k = L.kpo_spread_replicas(case["num"], tcs, n, init, ni, w.s(DISP["uids"][case["uid"]]), out, 64)
    got = [(out[i].name.ptr[:out[i].name.len].decode(), out[i].replicas) for i in range(k)]
    assert any(multiset_eq(got, [tuple(x) for x in want]) for want in case["wants"]), got


def test_fnv_parity():
    """UID parity used by tieBreakerByUID (binding.go:117-144; binding_test.go:55-57)."""
    L = O.lib()
    for uid, odd in ((DISP["uids"]["even"], 0), (DISP["uids"]["odd"], 1)):
        b = uid.encode()
        assert L.kpo_fnv32a(b, len(b)) & 1 == odd


# --------------------------------------------------------------------------- assignment
ASG = load("assign.json")


def run_assign(case, strategies):
    L = O.lib()
    w = api.World()
    cands = case["candidates"]
    clusters = [{"name": nm} for nm, _ in cands]
    ca, nc = w.clusters(clusters)
    cs = (O.kpo_candidate * max(1, len(cands)))(*[
        O.kpo_candidate(w.s(nm), 0, 0, 0, alloc, i) for i, (nm, alloc) in enumerate(cands)])
    spec = {"uid": "", "replicas": case["replicas"], "clusters": [{"name": a, "replicas": b} for a, b in case.get("clusters", [])],
            "placement": {}}
    fn = case["fn"]
    if fn == "static":
        rs = {"replicaSchedulingType": "Divided", "replicaDivisionPreference": "Weighted"}
        if case.get("weightPreference") is not None:
            rs["weightPreference"] = case["weightPreference"]
        spec["placement"]["replicaScheduling"] = rs
    elif fn in ("dynamic", "dynamic_scale_up"):
        spec["replicaRequirements"] = {"resourceRequest": {}}
        spec["placement"]["replicaScheduling"] = strategies[case["strategy"]]
    elif fn == "duplicated":
        spec["placement"]["replicaScheduling"] = None
    b = w.binding(spec)
    level = 2 if fn == "dynamic_scale_up" else 1
    ec, ea = C.c_int32(), C.c_int64()
    out = (api.kp_target_cluster * 64)()
    k = L.kpo_assign_replicas(cs, len(cands), ca, nc, C.byref(b), level, C.byref(ec), C.byref(ea), out, 64)
    if k < 0:
        return None, -k, ec.value
    got = [(out[i].name.ptr[:out[i].name.len].decode(), out[i].replicas) for i in range(k)]
    return got, 0, ec.value


@pytest.mark.parametrize("case", ASG["cases"], ids=ids(ASG["cases"]))
def test_assign(case):
    got, status, err = run_assign(case, ASG["strategies"])
    if case.get("wantErr"):
        assert got is None
        if case.get("errClass") == "unschedulable":
            assert status == api.STATUS_UNSCHEDULABLE
        return
    assert got is not None, (status, err)
    wants = case.get("wants") or [case["want"]]
    assert any(multiset_eq(got, [tuple(x) for x in want]) for want in wants), got


# --------------------------------------------------------------------------- selectors
SEL = load("selector.json")


@pytest.mark.parametrize("case", SEL["cases"], ids=ids(SEL["cases"]))
def test_cluster_matches(case):
    L = O.lib()
    w = api.World()
    c = w.cluster(SEL["cluster"])
    a = w.affinity(case["affinity"])
    assert L.kpo_cluster_matches(C.byref(c), C.byref(a)) == int(case["want"])


@pytest.mark.parametrize("case", SEL["zoneCases"], ids=ids(SEL["zoneCases"]))
def test_match_zones(case):
    L = O.lib()
    w = api.World()
    c = w.cluster({"name": "c", "zones": case["zones"]})
    a = w.affinity({"fieldSelector": {"matchExpressions": [case["expr"]]}})
    assert L.kpo_cluster_matches(C.byref(c), C.byref(a)) == int(case["want"])


# --------------------------------------------------------------------------- estimator
EST = load("estimator.json")
O.lib().kpo_estimator_part.argtypes = [C.POINTER(api.kp_cluster), C.POINTER(api.kp_binding),
                                       C.POINTER(api.kp_options), C.c_int, C.c_int, C.POINTER(C.c_int64)]


def _expand(v):
    if isinstance(v, str) and v.startswith("$"):
        return EST[v[1:]]
    if isinstance(v, dict):
        return {k: _expand(x) for k, x in v.items()}
    return v


@pytest.mark.parametrize("mode", [O.FAITHFUL, O.FAST])
@pytest.mark.parametrize("case", EST["cases"], ids=ids(EST["cases"]))
def test_estimator(case, mode):
    L = O.lib()
    w = api.World()
    c = w.cluster(_expand(case["cluster"]))
    spec = {"replicas": 1}
    if case.get("request") is not None:
        spec["replicaRequirements"] = {"resourceRequest": case["request"]}
    b = w.binding(spec)
    part = {"max": 0, "models": 1, "summary": 2, "allowed": 3}[case["fn"]]
    out = C.c_int64()
    opts = api.options(models_gate=case.get("modelsGate", True))
    rc = L.kpo_estimator_part(C.byref(c), C.byref(b), C.byref(opts), part, mode, C.byref(out))
    if case.get("expectError"):
        assert rc != 0
    else:
        assert rc == 0
    assert out.value == case["expected"]
