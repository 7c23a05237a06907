"""Reference spread-selection tests (tests/golden/spread.json, transcribed from
pkg/scheduler/core/spreadconstraint/*_test.go) through the oracle's unit hooks,
and selectGroups also through the engine's device restatement
(select_groups_dev, run by the host build libkp_cpusim.so).
"""
import ctypes as C
import json
import os

import pytest

import oracle_lib as O
from karmada_amd import api
from karmada_amd.engine import PKG

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SP = json.load(open(os.path.join(GOLDEN, "spread.json")))
L = O.lib()
L.kpo_sort_clusters.argtypes = [C.POINTER(O.kpo_candidate), C.c_uint32, C.c_int, C.POINTER(C.c_uint32)]
L.kpo_group_clusters.argtypes = [C.POINTER(api.kp_cluster), C.POINTER(C.c_int64), C.c_uint32, C.POINTER(api.kp_binding),
                                 C.c_int32, C.POINTER(C.c_uint32), C.POINTER(C.c_int32)]
L.kpo_select_by_region.argtypes = [C.POINTER(api.kp_str), C.POINTER(C.c_int64), C.POINTER(C.c_uint32), C.c_uint32,
                                   C.POINTER(O.kpo_candidate), C.c_int64, C.c_int64, C.c_int64, C.c_int64,
                                   C.POINTER(C.c_uint32)]
L.kpo_select_best.argtypes = [C.POINTER(O.kpo_candidate), C.c_uint32, C.POINTER(api.kp_binding), C.c_int32,
                              C.POINTER(C.c_uint32)]


def ids(cases):
    return [c["name"] for c in cases]


def cands(w, infos):
    arr = (O.kpo_candidate * max(1, len(infos)))(*[
        O.kpo_candidate(w.s(d["name"]), d["score"], d.get("ovf", 0), d["avail"], 0, -1) for d in infos])
    return arr


@pytest.mark.parametrize("case", SP["select_groups"], ids=ids(SP["select_groups"]))
def test_select_groups_oracle(case):
    w = api.World()
    g = case["groups"]
    names, n = w.arr(api.kp_str, [w.s(x["name"]) for x in g])
    vals = (C.c_int64 * max(1, n))(*[x["value"] for x in g])
    wts = (C.c_int64 * max(1, n))(*[x["weight"] for x in g])
    out = (C.c_uint32 * 64)()
    k = L.kpo_select_groups(names, vals, wts, n, case["min"], case["max"], case["target"], out)
    assert [g[out[i]]["name"] for i in range(k)] == case["expected"]


@pytest.mark.parametrize("case", SP["select_groups"], ids=ids(SP["select_groups"]))
def test_select_groups_device_code(case):
    """select_groups_dev (kp_paths.h): groups are regions with ids = name ranks."""
    S = C.CDLL(os.path.join(PKG, "libkp_cpusim.so"))
    S.kpsim_select_groups.argtypes = [C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.c_int, C.c_int64, C.c_int64,
                                      C.c_int64, C.POINTER(C.c_int32)]
    g = sorted(case["groups"], key=lambda x: x["name"])
    n = len(g)
    vals = (C.c_int32 * max(1, n))(*[x["value"] for x in g])
    wts = (C.c_int64 * max(1, n))(*[x["weight"] for x in g])
    out = (C.c_int32 * 64)()
    k = S.kpsim_select_groups(vals, wts, n, case["min"], case["max"], case["target"], out)
    got = [g[out[i]]["name"] for i in range(k)] if k > 0 else []
    assert got == case["expected"]


@pytest.mark.parametrize("case", SP["select_by_region"], ids=ids(SP["select_by_region"]))
def test_select_by_region_oracle(case):
    w = api.World()
    regs = case["regions"]
    flat, off = [], [0]
    for r in regs:
        flat += r["clusters"]
        off.append(len(flat))
    names, nr = w.arr(api.kp_str, [w.s(r["name"]) for r in regs])
    scores = (C.c_int64 * max(1, nr))(*[r["score"] for r in regs])
    offs = (C.c_uint32 * (nr + 1))(*off)
    out = (C.c_uint32 * 64)()
    k = L.kpo_select_by_region(names, scores, offs, nr, cands(w, flat), case["region"][0], case["region"][1],
                               case["cluster"][0], case["cluster"][1], out)
    if case["wantErr"]:
        assert k < 0
    else:
        assert k >= 0 and [flat[out[i]]["name"] for i in range(k)] == case["want"]


@pytest.mark.parametrize("case", SP["select_best"], ids=ids(SP["select_best"]))
def test_select_best_oracle(case):
    w = api.World()
    b = w.binding(case["binding"])
    out = (C.c_uint32 * 64)()
    cl = case["clusters"]
    k = L.kpo_select_best(cands(w, cl), len(cl), C.byref(b), case["need"], out)
    if case["wantErr"]:
        assert k < 0
    else:
        assert [cl[out[i]]["name"] for i in range(k)] == case["want"]


@pytest.mark.parametrize("case", SP["group_clusters"], ids=ids(SP["group_clusters"]))
def test_group_clusters_oracle(case):
    w = api.World()
    cs = [x["cluster"] for x in case["clusters"]]
    ca, n = w.clusters(cs)
    sc = (C.c_int64 * n)(*[x["score"] for x in case["clusters"]])
    b = w.binding(case["binding"])
    order = (C.c_uint32 * n)()
    groups = (C.c_int32 * 3)()
    assert L.kpo_group_clusters(ca, sc, n, C.byref(b), case["avail"], order, groups) == n
    assert [cs[order[i]]["name"] for i in range(n)] == case["order"]
    assert list(groups) == [case["zones"], case["regions"], case["providers"]]


@pytest.mark.parametrize("case", SP["calc_group_score"], ids=ids(SP["calc_group_score"]))
def test_calc_group_score_oracle(case):
    w = api.World()
    b = w.binding(case["binding"])
    s1 = L.kpo_calc_group_score(cands(w, case["a"]), len(case["a"]), C.byref(b), case["minGroups"])
    s2 = L.kpo_calc_group_score(cands(w, case["b"]), len(case["b"]), C.byref(b), case["minGroups"])
    assert (s1 >= s2) == case["aWins"]


@pytest.mark.parametrize("case", SP["calc_group_score_dup"], ids=ids(SP["calc_group_score_dup"]))
def test_calc_group_score_duplicate_oracle(case):
    w = api.World()
    b = w.binding(case["binding"])
    cl = case["clusters"]
    assert L.kpo_calc_group_score(cands(w, cl), len(cl), C.byref(b), 0) == case["score"]


@pytest.mark.parametrize("case", SP["sort_clusters"], ids=ids(SP["sort_clusters"]))
def test_sort_clusters_oracle(case):
    w = api.World()
    inf = case["infos"]
    order = (C.c_uint32 * max(1, len(inf)))()
    L.kpo_sort_clusters(cands(w, inf), len(inf), int(case["withAvail"]), order)
    assert [inf[order[i]]["name"] for i in range(len(inf))] == case["want"]
    if case["withAvail"]:  # the engine's sortClusters key (kp_algo.h sort_key) orders them the same
        keys = sorted(range(len(inf)), key=lambda i: (inf[i]["ovf"], -inf[i]["score"], -inf[i]["avail"],
                                                      inf[i]["name"]))
        assert [inf[i]["name"] for i in keys] == case["want"]


# ---- the engine's spread device code over the same tables (libkp_spreadtest.so) ----
# kp_paths.h's calcGroupScore (region_a_fast / region_a), selectGroups
# (select_groups_dev), selectBestClustersByRegion (region_b) and
# selectBestClustersByCluster (sel_cluster_fast), fed the tables' ClusterDetailInfo
# lists with their scores as sortClusters keys. gpu=0 runs them on the host (CpuBlk,
# the CPU suite), gpu=1 on gfx950 (one 256-thread workgroup, GpuBlk).
SPREADTEST = os.path.join(PKG, "libkp_spreadtest.so")


class KpstCand(C.Structure):
    _fields_ = [("rank", C.c_uint32), ("score", C.c_int32), ("ovf", C.c_int32), ("group", C.c_int32),
                ("avail", C.c_int64), ("alloc", C.c_int32), ("pad", C.c_int32)]


def spreadtest():
    S = C.CDLL(SPREADTEST)
    P = C.POINTER
    S.kpst_group_score.argtypes = [C.c_int, C.c_int, P(KpstCand), C.c_int, C.c_int, C.c_int32, C.c_int, C.c_int64,
                                   C.c_int64, P(C.c_int64), P(C.c_int32)]
    S.kpst_select_groups.argtypes = [C.c_int, P(C.c_int32), P(C.c_int64), C.c_int, C.c_int64, C.c_int64, C.c_int64,
                                     P(C.c_int32)]
    S.kpst_select_region.argtypes = [C.c_int, P(KpstCand), C.c_int, C.c_int, P(C.c_int64), C.c_int64, C.c_int64,
                                     C.c_int64, C.c_int64, P(C.c_uint32)]
    S.kpst_select_cluster.argtypes = [C.c_int, P(KpstCand), C.c_int, C.c_int64, C.c_int64, C.c_int32, P(C.c_uint32)]
    S.kpst_sort.argtypes = [C.c_int, P(KpstCand), C.c_int, P(C.c_uint32)]
    S.kpst_sort_key.restype = C.c_uint64
    S.kpst_sort_key.argtypes = [C.c_int32, C.c_int64, C.c_int64, C.c_uint32]
    S.kpst_key_fields.argtypes = [C.c_uint64, P(C.c_int32), P(C.c_int64), P(C.c_int64), P(C.c_uint32)]
    return S


def kcands(infos, groups=None):
    """The case's clusters renumbered by name (the engine's rank = name order)."""
    names = sorted({d["name"] for d in infos})
    rank = {n: i for i, n in enumerate(names)}
    arr = (KpstCand * max(1, len(infos)))()
    for i, d in enumerate(infos):
        arr[i] = KpstCand(rank[d["name"]], d["score"], d.get("ovf", 0), groups[i] if groups else 0, d["avail"],
                          d.get("alloc", d["avail"]), 0)
    return arr, names


def is_dup(binding):
    rs = (binding.get("placement") or {}).get("replicaScheduling")
    return not binding.get("placement") or rs is None or rs.get("replicaSchedulingType") == "Duplicated"


def device_group_score(S, gpu, walk, infos, binding, min_groups):
    arr, _ = kcands(infos)
    sc = (C.c_int64 * 1)()
    cn = (C.c_int32 * 1)()
    cmin = 0
    for s in (binding.get("placement") or {}).get("spreadConstraints") or []:
        if s["spreadByField"] == "cluster":
            cmin = s["minGroups"]
    rc = S.kpst_group_score(gpu, walk, arr, len(infos), 1, binding.get("replicas", 0), int(is_dup(binding)),
                            min_groups, cmin, sc, cn)
    assert rc == 0, rc
    assert cn[0] == len(infos)
    return sc[0]


def oracle_group_score(infos, binding, min_groups):
    w = api.World()
    b = w.binding(binding)
    return L.kpo_calc_group_score(cands(w, infos), len(infos), C.byref(b), min_groups)


# calcGroupScore with minGroups = 0 on a Divided binding (SURVEY hazard H4,
# group_clusters.go:248-249: ceil(Replicas / 0) = +Inf, converted to MinInt64 on amd64,
# so target*1000 wraps): the tables' lists again with Divided strategies and
# MinGroups 0, 1 and 3, and Replicas 0 (NaN -> MinInt64) — device code vs oracle.
H4_BINDINGS = [
    {"replicas": 100, "placement": {"replicaScheduling": {"replicaSchedulingType": "Divided",
                                                          "replicaDivisionPreference": "Aggregated"}}},
    {"replicas": 0, "placement": {"replicaScheduling": {"replicaSchedulingType": "Divided",
                                                        "replicaDivisionPreference": "Aggregated"}}},
    {"replicas": 55, "placement": {"replicaScheduling": {"replicaSchedulingType": "Divided",
                                                         "replicaDivisionPreference": "Weighted",
                                                         "weightPreference": {"dynamicWeight": "AvailableReplicas"}},
                                   "spreadConstraints": [{"spreadByField": "cluster", "minGroups": 2,
                                                          "maxGroups": 4}]}},
]


def group_score_cases():
    out = []
    for case in SP["calc_group_score"]:
        for side in ("a", "b"):
            out.append((f"{case['name']}/{side}", case[side], case["binding"], case["minGroups"]))
    for case in SP["calc_group_score_dup"]:
        out.append((case["name"], case["clusters"], case["binding"], 0))
    for case in SP["calc_group_score"]:
        for j, b in enumerate(H4_BINDINGS):
            for mg in (0, 1, 3):
                out.append((f"H4 {case['name']} b{j} min{mg}", case["a"], b, mg))
    return out


GS = group_score_cases()


def run_group_scores(gpu):
    S = spreadtest()
    bad = []
    for name, infos, binding, mg in GS:
        want = oracle_group_score(infos, binding, mg)
        for walk in (0, 1):
            got = device_group_score(S, gpu, walk, infos, binding, mg)
            if got != want:
                bad.append((name, walk, got, want))
    assert not bad, bad[:6]
    # the golden verdicts themselves (a's score >= b's)
    for case in SP["calc_group_score"]:
        a = device_group_score(S, gpu, 0, case["a"], case["binding"], case["minGroups"])
        b = device_group_score(S, gpu, 0, case["b"], case["binding"], case["minGroups"])
        assert (a >= b) == case["aWins"], case["name"]
    for case in SP["calc_group_score_dup"]:
        assert device_group_score(S, gpu, 1, case["clusters"], case["binding"], 0) == case["score"]


def run_select_groups(gpu):
    S = spreadtest()
    for case in SP["select_groups"]:
        g = sorted(case["groups"], key=lambda x: x["name"])
        n = len(g)
        vals = (C.c_int32 * max(1, n))(*[x["value"] for x in g])
        wts = (C.c_int64 * max(1, n))(*[x["weight"] for x in g])
        out = (C.c_int32 * 64)()
        k = S.kpst_select_groups(gpu, vals, wts, n, case["min"], case["max"], case["target"], out)
        got = [g[out[i]]["name"] for i in range(k)] if k > 0 else []
        assert got == case["expected"], case["name"]


def run_select_region(gpu):
    S = spreadtest()
    for case in SP["select_by_region"]:
        regs = sorted(case["regions"], key=lambda r: r["name"])
        infos, groups = [], []
        for gi, r in enumerate(regs):
            for cl in r["clusters"]:
                infos.append(cl)
                groups.append(gi)
        arr, names = kcands(infos, groups)
        scores = (C.c_int64 * len(regs))(*[r["score"] for r in regs])
        out = (C.c_uint32 * 64)()
        k = S.kpst_select_region(gpu, arr, len(infos), len(regs), scores, case["region"][0], case["region"][1],
                                 case["cluster"][0], case["cluster"][1], out)
        if case["wantErr"]:
            assert k < 0, case["name"]
        else:
            assert k >= 0 and [names[out[i]] for i in range(k)] == case["want"], case["name"]


def run_select_best(gpu):
    """SelectBestClusters (select_clusters.go:28-80): the dispatch the packer makes
    (h.sel, h.need_replicas), then the device selection."""
    S = spreadtest()
    for case in SP["select_best"]:
        p = case["binding"].get("placement") or {}
        rs = p.get("replicaScheduling")
        scs = p.get("spreadConstraints") or []
        wp = (rs or {}).get("weightPreference")
        ignore_spread = bool(rs and rs.get("replicaSchedulingType") == "Divided" and
                             rs.get("replicaDivisionPreference") == "Weighted" and
                             (wp is None or (wp.get("staticWeightList") and not wp.get("dynamicWeight"))))
        need = -1 if (rs is None or rs.get("replicaSchedulingType") == "Duplicated") else case["need"]
        cl = case["clusters"]
        arr, names = kcands(cl)
        out = (C.c_uint32 * 64)()
        fields = {s["spreadByField"]: s for s in scs}
        if not scs or ignore_spread:
            k = S.kpst_sort(gpu, arr, len(cl), out)  # "select all": the sorted candidates
        else:
            assert "region" not in fields  # (the table holds cluster constraints only)
            c = fields["cluster"]
            k = S.kpst_select_cluster(gpu, arr, len(cl), c["minGroups"], c["maxGroups"], need, out)
        if case["wantErr"]:
            assert k < 0, case["name"]
        else:
            assert [names[out[i]] for i in range(k)] == case["want"], case["name"]


def run_sort_clusters(gpu):
    S = spreadtest()
    for case in SP["sort_clusters"]:
        if not case["withAvail"]:
            continue  # (sortClusters without the AvailableReplicas compare: not the engine's key)
        inf = case["infos"]
        arr, names = kcands(inf)
        out = (C.c_uint32 * max(1, len(inf)))()
        k = S.kpst_sort(gpu, arr, len(inf), out)
        assert [names[out[i]] for i in range(k)] == case["want"], case["name"]


def test_sort_key_fields_roundtrip():
    """The 7-bit score field (0..100 framework scores), overflow orders up to
    kMaxOvfTerms - 1 and 1000, AvailableReplicas over [-2^32, 2^32), rank 18 bits;
    ascending keys = (OverflowOrder asc, Score desc, AvailableReplicas desc, Name asc)."""
    import random
    S = spreadtest()
    rng = random.Random(5)
    recs = []
    for _ in range(3000):
        ovf = rng.choice([0, 0, 1, 2, 61, 62, 1000])
        score = rng.choice([0, 100, rng.randint(0, 100)])
        avail = rng.choice([0, 1, -1, 2**31 - 1, -2**31, 2**32 - 2, -2**32, rng.randint(-2**32, 2**32 - 1)])
        rank = rng.randint(0, 2**18 - 1)
        k = S.kpst_sort_key(ovf, score, avail, rank)
        o, s, a, r = C.c_int32(), C.c_int64(), C.c_int64(), C.c_uint32()
        S.kpst_key_fields(k, C.byref(o), C.byref(s), C.byref(a), C.byref(r))
        assert (o.value, s.value, a.value, r.value) == (ovf, score, avail, rank)
        recs.append((k, (ovf, -score, -avail, rank)))
    assert sorted(recs, key=lambda x: x[0]) == sorted(recs, key=lambda x: x[1])


@pytest.mark.parametrize("table", ["group_score", "select_groups", "select_region", "select_best", "sort"])
def test_spread_tables_device_code_host(table):
    {"group_score": run_group_scores, "select_groups": run_select_groups, "select_region": run_select_region,
     "select_best": run_select_best, "sort": run_sort_clusters}[table](0)


@pytest.mark.gpu
@pytest.mark.parametrize("table", ["group_score", "select_groups", "select_region", "select_best", "sort"])
def test_spread_tables_device_code_gpu(table):
    {"group_score": run_group_scores, "select_groups": run_select_groups, "select_region": run_select_region,
     "select_best": run_select_best, "sort": run_sort_clusters}[table](1)
