"""The bitset filter (kp_filter.h: k_filter, the schedule path's default filter
stage) against the per-pair evaluator (k_pair, KP_PAIR_ROWS=1) and the oracle.

- The reference's own ClusterMatches / matchZones tables (tests/golden/selector.json,
  pkg/util/selector_test.go) through kp_filter_batch with only ClusterAffinity
  enabled, in both modes.
- Seeded universes whose selectors use every selector opcode the packer emits:
  label In/NotIn/Exists/DoesNotExist and matchLabels, provider/region field
  In/NotIn/Exists/DoesNotExist/Gt/Lt, zone In/NotIn/Exists/DoesNotExist, cluster
  names and excludes, several affinity terms, spec.Clusters (TargetContains),
  eviction tasks, tolerations, GVKs and spread-constraint presence; the feasibility
  of every (binding, cluster) pair equals the oracle's RunFilterPlugins
  (kpo_filter) in both modes.
"""
import ctypes as C
import json
import os
import random

import pytest

import oracle_lib as O
from karmada_amd import api

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SEL = json.load(open(os.path.join(GOLDEN, "selector.json")))


def _filter(engine, clusters, bindings, opts, rows):
    from karmada_amd.engine import GenericScheduler
    if rows:
        os.environ["KP_PAIR_ROWS"] = "1"
    try:
        g = GenericScheduler(engine, clusters, opts)
        return g.filter(bindings)
    finally:
        os.environ.pop("KP_PAIR_ROWS", None)


def _selector_cases():
    out = []
    for c in SEL["cases"]:
        out.append((c["name"], SEL["cluster"], c["affinity"], c["want"]))
    for c in SEL["zoneCases"]:
        out.append(("zone: " + c["name"], {"name": "c", "zones": c["zones"]},
                    {"fieldSelector": {"matchExpressions": [c["expr"]]}}, c["want"]))
    return out


CASES = _selector_cases()


def _check_golden(engine, rows):
    opts = api.options(plugins=api.PLUGIN_CLUSTER_AFFINITY)
    bad = []
    for name, cluster, aff, want in CASES:
        got = _filter(engine, [cluster], [{"placement": {"clusterAffinity": aff}}], opts, rows)[0]
        if (got == [cluster["name"]]) != want:
            bad.append(name)
    assert not bad, bad


@pytest.mark.parametrize("rows", [False, True], ids=["bits", "rows"])
def test_selector_golden_cpusim(cpusim_engine, rows):
    _check_golden(cpusim_engine, rows)


# ---------------------------------------------------------------- seeded universes
KEYS = ["env", "tier", "team", "gpu"]
VALS = ["a", "b", "c", "d", "e"]
PROV = ["aws", "gcp", "12", "7", "-3"]
REGS = ["r1", "r2", "100", "5"]
ZONES = ["z1", "z2", "z3", "z4"]
GVKS = [("apps/v1", "Deployment"), ("batch/v1", "Job"), ("v1", "Service")]


def _cluster(r, i):
    d = {"name": "m-%04d" % i, "labels": {}}
    for k in KEYS:
        if r.random() < 0.7:
            d["labels"][k] = r.choice(VALS)
    if r.random() < 0.85:
        d["provider"] = r.choice(PROV)
    if r.random() < 0.85:
        d["region"] = r.choice(REGS)
    if r.random() < 0.8:
        d["zones"] = r.sample(ZONES, r.randint(1, 3))
    if r.random() < 0.3:
        d["taints"] = [{"key": r.choice(["dedicated", "maint"]), "value": r.choice(["gpu", "x"]),
                        "effect": r.choice(["NoSchedule", "NoExecute", "PreferNoSchedule"])}]
    d["apiEnablements"] = [{"groupVersion": gv, "resources": [{"kind": k}]}
                           for gv, k in GVKS if r.random() < 0.9]
    d["deleting"] = r.random() < 0.05
    return d


def _req(r, key, vals):
    op = r.choice(["In", "NotIn", "Exists", "DoesNotExist"])
    e = {"key": key, "operator": op}
    if op in ("In", "NotIn"):
        e["values"] = r.sample(vals, r.randint(1, 3)) + (["nope"] if r.random() < 0.2 else [])
    return e


def _affinity(r, names):
    a = {}
    if r.random() < 0.7:
        ls = {}
        if r.random() < 0.4:
            ls["matchLabels"] = {r.choice(KEYS): r.choice(VALS)}
        ls["matchExpressions"] = [_req(r, r.choice(KEYS + ["absent"]), VALS) for _ in range(r.randint(0, 2))]
        a["labelSelector"] = ls
    if r.random() < 0.5:
        ex = []
        for _ in range(r.randint(1, 2)):
            f = r.choice(["provider", "region", "zone"])
            if f == "zone":
                ex.append(_req(r, "zone", ZONES))
            elif r.random() < 0.3:
                ex.append({"key": f, "operator": r.choice(["Gt", "Lt"]), "values": [str(r.randint(-5, 20))]})
            else:
                ex.append(_req(r, f, PROV if f == "provider" else REGS))
        a["fieldSelector"] = {"matchExpressions": ex}
    if r.random() < 0.15:
        a["clusterNames"] = r.sample(names, min(len(names), r.randint(1, 8)))
    if r.random() < 0.15:
        a["exclude"] = r.sample(names, min(len(names), r.randint(1, 8)))
    return a


def _binding(r, names):
    gv, k = r.choice(GVKS + [("nope/v9", "Thing")])
    p = {}
    if r.random() < 0.6:
        p["clusterAffinity"] = _affinity(r, names)
    elif r.random() < 0.5:
        terms = [dict(_affinity(r, names), affinityName="t%d" % j) for j in range(r.randint(1, 3))]
        p["clusterAffinities"] = terms
    if r.random() < 0.5:
        p["clusterTolerations"] = [{"key": "dedicated", "operator": r.choice(["Equal", "Exists"]), "value": "gpu",
                                    "effect": r.choice(["", "NoSchedule"])}]
    if r.random() < 0.2:
        p["spreadConstraints"] = [{"spreadByField": r.choice(["provider", "region", "zone"]), "maxGroups": 2,
                                   "minGroups": 1}]
    d = {"apiVersion": gv, "kind": k, "replicas": 3, "placement": p,
         "schedulerObservedAffinityName": "t%d" % r.randint(0, 3)}
    if r.random() < 0.2:
        d["clusters"] = [{"name": n, "replicas": 1} for n in r.sample(names, min(len(names), r.randint(1, 4)))]
    if r.random() < 0.1:
        d["gracefulEvictionTasks"] = [{"fromCluster": n} for n in r.sample(names, min(len(names), 2))]
    return d


def _universe(seed, nc, nb):
    r = random.Random(seed)
    clusters = [_cluster(r, i) for i in range(nc)]
    names = [c["name"] for c in clusters]
    return clusters, [_binding(r, names) for _ in range(nb)]


def _oracle(clusters, bindings, opts):
    w = api.World()
    L = O.lib()
    cs = [w.cluster(c) for c in clusters]
    out = []
    for d in bindings:
        b = w.binding(d)
        out.append([clusters[i]["name"] for i, c in enumerate(cs)
                    if not clusters[i].get("deleting") and L.kpo_filter(C.byref(c), C.byref(b), C.byref(opts)) == 0])
    return out


UNIVERSES = [(1, 70, 200), (2, 130, 150), (3, 1, 40), (4, 64, 120), (5, 200, 100)]


def _check_universe(engine, seed, nc, nb, rows):
    clusters, bindings = _universe(seed, nc, nb)
    opts = api.options()
    got = _filter(engine, clusters, bindings, opts, rows)
    want = _oracle(clusters, bindings, opts)
    bad = [i for i in range(nb) if sorted(got[i]) != sorted(want[i])]
    assert not bad, (len(bad), bad[0], sorted(got[bad[0]]), sorted(want[bad[0]]), bindings[bad[0]])


@pytest.mark.parametrize("rows", [False, True], ids=["bits", "rows"])
@pytest.mark.parametrize("seed,nc,nb", UNIVERSES)
def test_filter_universe_cpusim(cpusim_engine, seed, nc, nb, rows):
    _check_universe(cpusim_engine, seed, nc, nb, rows)


@pytest.mark.gpu
def test_selector_golden_gpu(gpu_engine):
    _check_golden(gpu_engine, False)
    _check_golden(gpu_engine, True)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,nc,nb", UNIVERSES + [(6, 700, 300), (7, 5000, 60)])
def test_filter_universe_gpu(gpu_engine, seed, nc, nb):
    _check_universe(gpu_engine, seed, nc, nb, False)
    _check_universe(gpu_engine, seed, nc, nb, True)
