"""The per-pair plugin and estimator interfaces the Go shim of INTEGRATION.md exposes,
through their Python mirror (karmada_amd/plugins.py) over the engine's CPU build:

- runtime.Registry and `--plugins` (registry_test.go tables, tests/golden/util_binding.json)
  and the enabled_plugins bitmask they produce;
- frameworkImpl's RunFilterPlugins / RunScorePlugins loops with stub plugins, as
  framework_test.go:32 and :114 drive them with gomock (those tables' rows restated
  below: a stub per mock behaviour, the expected IsSuccess per row);
- KpFilter / KpScore answering Filter / Score per (binding slot, cluster) from one
  batch, and KpEstimator answering MaxAvailableReplicas in the request's cluster order,
  each against the oracle's per-pair restatement.
"""
import ctypes as C
import json
import os

import pytest

from karmada_amd import api, plugins, synth
from karmada_amd.engine import Batch, Snapshot
import oracle_lib as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
with open(os.path.join(GOLDEN, "util_binding.json")) as f:
    REG = json.load(f)["registry"]


@pytest.mark.parametrize("case", REG["filter"], ids=lambda c: c["name"] + " " + ",".join(c["curPlugins"]))
def test_registry_filter(case):
    r = plugins.Registry()
    for n in case["registered"]:
        r.register(n, object)
    assert r.filter(case["curPlugins"]).factory_names() == case["expectedPlugins"]


@pytest.mark.parametrize("case", REG["register"], ids=lambda c: c["name"])
def test_registry_register(case):
    r = plugins.Registry()
    for n in case["initialPlugins"]:
        r.register(n, object)
    try:
        r.register(case["plugin"], object)
        err = False
    except ValueError:
        err = True
    assert err == case["wantErr"] and r.factory_names() == case["expectedPlugins"]


@pytest.mark.parametrize("case", REG["unregister"], ids=lambda c: c["name"])
def test_registry_unregister(case):
    r = plugins.Registry()
    for n in case["initialPlugins"]:
        r.register(n, object)
    try:
        r.unregister(case["plugin"])
        err = False
    except ValueError:
        err = True
    assert err == case["wantErr"] and r.factory_names() == case["expectedPlugins"]


@pytest.mark.parametrize("flags,mask", [
    (["*"], api.PLUGIN_ALL),
    (["*", "-TaintToleration"], api.PLUGIN_ALL & ~api.PLUGIN_TAINT_TOLERATION),
    (["-ClusterLocality", "*"], api.PLUGIN_ALL & ~api.PLUGIN_CLUSTER_LOCALITY),  # '*' applies first
    (["-ClusterAffinity", "ClusterAffinity"], api.PLUGIN_CLUSTER_AFFINITY),  # '-x' before any enable: no effect
    (["ClusterAffinity", "APIEnablement"], api.PLUGIN_CLUSTER_AFFINITY | api.PLUGIN_API_ENABLEMENT),
    (["*", "-APIEnablement", "-TaintToleration", "-ClusterAffinity", "-SpreadConstraint", "-ClusterEviction",
      "-ClusterLocality"], 0),
])
def test_enabled_plugins_mask(flags, mask, cpusim_engine):
    """--plugins -> kp_options.enabled_plugins, and the engine scheduling with it agrees
    with the oracle run with the same enabled set."""
    assert plugins.enabled_plugins_mask(flags) == mask
    u = synth.Universe(6, 41, 80, 0, 300)
    opts = api.options(plugins=mask)
    snap = Snapshot.from_structs(cpusim_engine, u.clusters, u.n_clusters, u.names, opts)
    b = Batch(snap, structs=u.binding_slice(0, u.n_bindings))
    got = b.schedule()
    b.close()
    snap.close()
    assert got == O.schedule_c(u.clusters, u.n_clusters, u.bindings, u.n_bindings, opts, O.FAST, 4)


# framework_test.go:32 (Test_frameworkImpl_RunFilterPlugins): mocks return Error("foo") or Success
class _Filter:
    def __init__(self, ok):
        self.ok = ok

    def name(self):
        return "foo"

    def filter(self, ctx):
        return plugins.Result(plugins.SUCCESS) if self.ok else plugins.Result(plugins.ERROR, "foo")


@pytest.mark.parametrize("name,stubs,success", [
    ("no filter plugin", [], True),
    ("error filter plugin", [False], False),
    ("success filter plugin", [True], True),
    ("error and success filter plugins", [False, True], False),
    ("success and error filter plugins", [True, False], False),
])
def test_run_filter_plugins(name, stubs, success):
    reg = plugins.Registry()
    for i, ok in enumerate(stubs):  # createAndRegisterFactory: foo0, foo1, ...
        reg.register("foo%d" % i, (lambda ok=ok: _Filter(ok)))
    r = plugins.Framework(reg).run_filter_plugins(None)
    assert plugins.is_success(r) == success


# framework_test.go:114 (Test_frameworkImpl_RunScorePlugins): Score (60, Success) or
# (-1, Error); NormalizeScore Success or Error
class _Norm:
    def __init__(self, ok):
        self.ok = ok

    def normalize_score(self, scores):
        return None if self.ok else plugins.Result(plugins.ERROR, "foo")


class _Score:
    def __init__(self, score_ok, norm_ok):
        self.score_ok, self.norm_ok = score_ok, norm_ok

    def name(self):
        return "foo"

    def score(self, spec, cluster):
        return (60, plugins.Result(plugins.SUCCESS)) if self.score_ok else (-1, plugins.Result(plugins.ERROR, "foo"))

    def score_extensions(self):
        return _Norm(self.norm_ok)


@pytest.mark.parametrize("name,score_ok,norm_ok,success", [
    ("Test score ok", True, True, True),
    ("Test score func error", False, True, False),
    ("Test normalize score error", True, False, False),
])
def test_run_score_plugins(name, score_ok, norm_ok, success):
    reg = plugins.Registry()
    reg.register("foo0", lambda: _Score(score_ok, norm_ok))
    scores, r = plugins.Framework(reg).run_score_plugins(None, ["c1"])
    assert plugins.is_success(r) == success
    assert (scores == {"foo": [("c1", 60)]}) == success


def test_kp_plugins_per_pair(cpusim_engine):
    """KpFilter / KpScore / KpEstimator, registered in a Framework in place of the
    in-tree plugins, answer every (binding, cluster) pair as the oracle's
    RunFilterPlugins / ScoreCluster / GeneralEstimator restatements do."""
    u = synth.Universe(6, 42, 70, 0, 120)
    opts = api.options()
    snap = Snapshot.from_structs(cpusim_engine, u.clusters, u.n_clusters, u.names, opts)
    b = Batch(snap, structs=u.binding_slice(0, u.n_bindings))
    def s(x):
        return C.string_at(x.ptr, x.len).decode() if x.len else ""
    taints = [{"taints": [{"key": s(t.key), "value": s(t.value), "effect": s(t.effect)}
                          for t in u.clusters[c].taints[:u.clusters[c].n_taints]]} for c in range(u.n_clusters)]
    view = plugins.BatchView(snap, b, taints)
    reg = plugins.Registry()
    reg.register("KpFilter", lambda: plugins.KpFilter(view))
    reg.register("KpScore", lambda: plugins.KpScore(view))
    fw = plugins.Framework(reg)
    est = plugins.KpEstimator(snap, b)
    OL = O.lib()
    order = list(reversed(u.names))  # the request's cluster order is kept
    bad = []
    for i in range(u.n_bindings):
        bp = C.pointer(u.bindings[i])
        scores, r = fw.run_score_plugins(i, u.names)
        assert r is None
        ests = dict(est.max_available_replicas(i, order))
        assert [n for n, _ in est.max_available_replicas(i, order)] == order
        for c, name in enumerate(u.names):
            cp = C.pointer(u.clusters[c])
            res = fw.run_filter_plugins((i, name))
            want_fit = OL.kpo_filter_reason(cp, bp, C.byref(opts)) & 0xFF in (api.REASON_FIT, api.REASON_DELETING)
            if plugins.is_success(res) != want_fit:
                bad.append(("filter", i, name, res))
            if scores["KpScore"][c][1] != OL.kpo_score(cp, bp, C.byref(opts)):
                bad.append(("score", i, name))
            if ests[name] != OL.kpo_max_available_replicas(cp, bp, C.byref(opts), O.FAST):
                bad.append(("estimate", i, name))
    b.close()
    snap.close()
    assert not bad, bad[:5]


def test_kp_estimator_component_sets(cpusim_engine):
    """MaxAvailableComponentSets through the estimator shim, request order kept, against
    the oracle's per-cluster restatement (general.go:163-292)."""
    u = synth.Universe(9, 43, 40, 0, 0)
    opts = api.options(multi_templates=True)
    snap = Snapshot.from_structs(cpusim_engine, u.clusters, u.n_clusters, u.names, opts)
    est = plugins.KpEstimator(snap, None)
    comps = [{"name": "a", "replicas": 2, "replicaRequirements": {"resourceRequest": {"cpu": "500m", "memory": "1Gi"}}},
             {"name": "b", "replicas": 1, "replicaRequirements": {"resourceRequest": {"cpu": "2"}}}]
    order = u.names[::3]
    got = est.max_available_component_sets(comps, order)
    assert [n for n, _ in got] == order
    w = api.World()
    ca, nc = w.components(comps)
    OL = O.lib()
    for n, sets in got:
        c = u.names.index(n)
        assert sets == OL.kpo_max_available_component_sets(C.pointer(u.clusters[c]), ca, nc, C.byref(opts), O.FAST)
    snap.close()


# ---- the shim's spec -> slot index and estimator cache (plugins.Shim) ----
APIS = [{"groupVersion": "apps/v1", "resources": [{"kind": "Deployment"}]}]


def shim_clusters(cpu=("4", "8", "2")):
    return [{"name": f"m{i}", "apiEnablements": APIS, "labels": {"env": "prod" if i % 2 == 0 else "dev"},
             "resourceSummary": {"allocatable": {"cpu": c, "memory": "64Gi", "pods": "100"},
                                 "allocated": {}, "allocating": {}}} for i, c in enumerate(cpu)]


def shim_spec(replicas=3, env=None):
    p = {"replicaScheduling": {"replicaSchedulingType": "Divided", "replicaDivisionPreference": "Weighted",
                               "weightPreference": {"dynamicWeight": "AvailableReplicas"}}}
    if env:
        p["clusterAffinity"] = {"labelSelector": {"matchLabels": {"env": env}}}
    return {"replicas": replicas, "replicaRequirements": {"resourceRequest": {"cpu": "1"}}, "placement": p,
            "clusters": [{"name": "m0", "replicas": 1}]}


def test_shim_spec_slot_lookup(cpusim_engine):
    """ScheduleBatch registers every spec it packs; Filter/Score for them are lookups
    (no batch packed); an unseen spec is packed once as a one-binding batch; the Go map
    is keyed by pointer, so an equal-content copy is a different spec."""
    sh = plugins.Shim(cpusim_engine, shim_clusters())
    a, b = shim_spec(env="prod"), shim_spec(env="dev")
    res = sh.schedule_batch([a, b])
    assert len(res) == 2 and sh.batches_created == 1
    for c in ("m0", "m1", "m2"):
        fa, fb = sh.filter(a, c), sh.filter(b, c)
        assert (fa is None) == (c in ("m0", "m2")) and (fb is None) == (c == "m1")
        assert sh.score(a, c)[0] == (100 if c == "m0" else 0)
    assert sh.batches_created == 1
    cold = shim_spec(env="prod")
    assert sh.filter(cold, "m0") is None and sh.batches_created == 2
    assert sh.filter(cold, "m1") is not None and sh.batches_created == 2
    sh.release([a, b, cold])
    assert not sh.by and not sh.live
    sh.close()


def test_shim_release_destroys_batches(cpusim_engine):
    sh = plugins.Shim(cpusim_engine, shim_clusters())
    a, b = shim_spec(), shim_spec()
    sh.schedule_batch([a, b])
    view = sh.by[id(a)][0]
    sh.release([a])
    assert view.batch.h  # b still holds the view
    sh.release([b])
    assert not view.batch.h
    sh.close()


def test_shim_estimator_cache_by_content(cpusim_engine):
    """MaxAvailableReplicas builds a one-binding batch per distinct ReplicaRequirements
    content and reuses it (the r3 shim packed a fresh spec on every call and never
    freed it); answers are the GeneralEstimator's (cpu allocatable / request)."""
    sh = plugins.Shim(cpusim_engine, shim_clusters())
    req = {"resourceRequest": {"cpu": "1"}}
    assert sh.max_available_replicas(req, ["m2", "m0", "m1"]) == [("m2", 2), ("m0", 4), ("m1", 8)]
    assert sh.max_available_replicas({"resourceRequest": {"cpu": "1"}}, ["m1"]) == [("m1", 8)]
    assert sh.batches_created == 1
    assert sh.max_available_replicas({"resourceRequest": {"cpu": "2"}}, ["m1", "m0"]) == [("m1", 4), ("m0", 2)]
    assert sh.batches_created == 2
    assert sh.max_available_replicas(None, ["m0"]) == [("m0", 100)]  # no requirements: allowed pods
    sh.close()


def test_shim_update_invalidates(cpusim_engine):
    """Cluster events re-pack the snapshot and drop every cached view: the next answers
    come from the new snapshot, never a stale batch."""
    sh = plugins.Shim(cpusim_engine, shim_clusters())
    req = {"resourceRequest": {"cpu": "1"}}
    a = shim_spec()
    sh.schedule_batch([a])
    assert sh.max_available_replicas(req, ["m0"]) == [("m0", 4)]
    sh.update(shim_clusters(cpu=("16", "8", "2"))[:1])
    assert not sh.by and not sh.est
    assert sh.max_available_replicas(req, ["m0"]) == [("m0", 16)]
    sh.close()


def test_shim_refuses_out_of_tree_plugins(cpusim_engine):
    """A registry with an out-of-tree score plugin: the batch path refuses (KP_ENOTSUP,
    kp_options.n_out_of_tree_plugins) instead of placing without that plugin's scores;
    the per-pair answers, which the framework combines with the other plugin, remain."""
    from karmada_amd.engine import EngineError
    names = list(plugins.IN_TREE) + ["KpPlacement", "MyScore"]
    assert plugins.out_of_tree_plugins(names) == 1
    sh = plugins.Shim(cpusim_engine, shim_clusters(), registry_names=names)
    a = shim_spec()
    with pytest.raises(EngineError, match="rc=-4"):
        sh.schedule_batch([a])
    assert sh.filter(a, "m0") is None
    sh.close()
    sh = plugins.Shim(cpusim_engine, shim_clusters(), registry_names=list(plugins.IN_TREE) + ["KpPlacement"])
    assert len(sh.schedule_batch([shim_spec()])) == 1
    sh.close()


def test_shim_estimator_view_skips_filter_and_score(cpusim_engine):
    """An estimator-only view (one binding per ReplicaRequirements content) answers
    MaxAvailableReplicas through kp_max_available_replicas alone: the per-pair
    filter-reason and score passes never run for it (every distinct
    request used to pay kp_filter_reasons + kp_score_batch over the whole snapshot)."""
    sh = plugins.Shim(cpusim_engine, shim_clusters())
    assert sh.max_available_replicas({"resourceRequest": {"cpu": "1"}}, ["m0", "m1"]) == [("m0", 4), ("m1", 8)]
    (view, _), = sh.est.values()
    assert view.passes == []
    # a Filter / Score view runs each pass once, on first use
    a = shim_spec(env="prod")
    sh.schedule_batch([a])
    va = sh.by[id(a)][0]
    assert va.passes == []
    sh.filter(a, "m0"), sh.filter(a, "m1")
    assert va.passes == ["kp_filter_reasons"]
    sh.score(a, "m0"), sh.score(a, "m2")
    assert va.passes == ["kp_filter_reasons", "kp_score_batch"]
    sh.close()


def test_shim_unknown_cluster_is_an_error(cpusim_engine):
    """A cluster name the snapshot does not hold (added since the last update) is an
    Error Result / exception, never the answer of cluster index 0 (a Go map's zero
    value)."""
    sh = plugins.Shim(cpusim_engine, shim_clusters())
    a = shim_spec(env="prod")
    sh.schedule_batch([a])
    r = sh.filter(a, "m9")
    assert r is not None and r.code == plugins.ERROR and "m9" in r.reasons[0]
    s, r = sh.score(a, "m9")
    assert s == 0 and r is not None and r.code == plugins.ERROR
    with pytest.raises(plugins.UnknownCluster):
        sh.max_available_replicas({"resourceRequest": {"cpu": "1"}}, ["m0", "m9"])
    est = plugins.KpEstimator(sh.snap, None)
    with pytest.raises(plugins.UnknownCluster):
        est.max_available_component_sets([{"name": "a", "replicas": 1}], ["nope"])
    sh.close()


def test_shim_empty_cluster_lists(cpusim_engine):
    """Empty request cluster lists answer an empty list (the Go shim's length guard
    before &idx[0])."""
    sh = plugins.Shim(cpusim_engine, shim_clusters(), opts=api.options(multi_templates=True))
    assert sh.max_available_replicas({"resourceRequest": {"cpu": "1"}}, []) == []
    est = plugins.KpEstimator(sh.snap, None)
    assert est.max_available_component_sets([{"name": "a", "replicas": 1}], []) == []
    sh.close()


def test_shim_keeps_callers_options(cpusim_engine):
    """The shim sets n_out_of_tree_plugins on a copy: the caller's kp_options object is
    unchanged and can build another snapshot without this shim's count."""
    opts = api.options()
    names = list(plugins.IN_TREE) + ["KpPlacement", "MyScore"]
    sh = plugins.Shim(cpusim_engine, shim_clusters(), opts=opts, registry_names=names)
    assert opts.n_out_of_tree_plugins == 0
    sh.close()
    sh = plugins.Shim(cpusim_engine, shim_clusters(), opts=opts)
    assert len(sh.schedule_batch([shim_spec()])) == 1
    sh.close()


def test_shim_keyed_batches_reuse_records(cpusim_engine):
    """ScheduleBatchKeyed: a second cycle over the same (uid, generation) reuses every
    packed record and schedules as a fresh pack; a bumped generation re-packs that one."""
    sh = plugins.Shim(cpusim_engine, shim_clusters())
    specs = [dict(shim_spec(env=e, replicas=r), uid="uid-%d" % i)
             for i, (e, r) in enumerate([("prod", 2), ("dev", 3), (None, 5), ("prod", 1)])]
    first = sh.schedule_batch(specs, generations=[1, 1, 1, 1])
    assert sh.pack_cache.stats()["last_hits"] == 0
    again = sh.schedule_batch(specs, generations=[1, 1, 1, 1])
    assert sh.pack_cache.stats()["last_hits"] == 4
    assert again == first == sh.schedule_batch(specs)
    sh.schedule_batch(specs, generations=[1, 2, 1, 1])
    assert sh.pack_cache.stats()["last_hits"] == 3
    sh.close()
