"""The reference's own assignment, division and Webster tables run through the WHOLE
engine (kp_schedule_batch: filter -> score -> GeneralEstimator -> select -> assign),
on the host build on every CPU run and on the MI355X in the -m gpu suite.

Each case becomes a snapshot plus one binding:
  * a case cluster's AvailableReplicas / AllocatableReplicas becomes its
    ResourceSummary's allocatable pods, and the binding carries no
    ReplicaRequirements, so the GeneralEstimator answers exactly that number
    (getAllowedPodNumber, estimator/client/general.go:57-108);
  * AvailableReplicas = AllocatableReplicas + the binding's spec.Clusters replicas, as
    the cases give them;
  * a Webster party or a Dispenser weight becomes a cluster of that name (its votes
    as allocatable pods for DynamicWeight; its weight as a StaticWeight rule for the
    Dispenser), the tie-breaker a binding UID of the matching FNV parity.
Schedule drops zero-replica targets (removeZeroReplicasCluster, core/common.go:153)
unless EnableEmptyWorkloadPropagation attaches every selected cluster
(generic_scheduler.go:109-111), so each case is checked both ways.

Cases a Schedule call cannot express are listed in NOT_EXPRESSIBLE with the reason.
Sources: core.json (generic_scheduler_test.go:36 Test_DistributionOfReplicas,
common_test.go TestAssignReplicas, division_algorithm_test.go
Test_dynamicDivideReplicas), webster.json (webstermethod_test.go:42
TestAllocateWebsterSeats), dispenser.json (util/helper/binding_test.go:60).
"""
import json
import os

import pytest

from karmada_amd import api
from karmada_amd.engine import PKG, Batch, Engine, Snapshot

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CORE = json.load(open(os.path.join(GOLDEN, "core.json")))
WEB = json.load(open(os.path.join(GOLDEN, "webster.json")))
DISP = json.load(open(os.path.join(GOLDEN, "dispenser.json")))
UIDS = DISP["uids"]  # "even" / "odd": FNV-1a parity of the UID (the Dispenser's tie order)

NOT_EXPRESSIBLE = {
    "core/assign/No clusters available":
        "an empty cluster list fails findClustersThatFit (FitError) before AssignReplicas' own error",
    "webster/empty party votes, expect nil result": "no parties = no clusters: FitError first",
    "webster/both party votes and newSeats are 0, expect nil result": "no parties = no clusters: FitError first",
    "webster/tie-breaker is nil, expect break tie by seats":
        "initial seats: dynamicDivideReplicas spreads with init=nil (division_algorithm.go:95)",
    "webster/non-initial allocation, new party joins, only new party gets new seats":
        "initial seats: dynamicDivideReplicas spreads with init=nil (division_algorithm.go:95)",
    "webster/non-initial allocation, both new and old parties compete for new seats":
        "initial seats: dynamicDivideReplicas spreads with init=nil (division_algorithm.go:95)",
    "webster/non-initial allocation, initialAssignments party not in partyVotes, expect no new seats for that party":
        "initial seats: dynamicDivideReplicas spreads with init=nil (division_algorithm.go:95)",
    "dispenser/Scale up 6 replicas": "init: assignByStaticWeightStrategy builds its Dispenser with init=nil (assignment.go:208)",
    "dispenser/Scale up 3 replicas": "init: assignByStaticWeightStrategy builds its Dispenser with init=nil (assignment.go:208)",
    "dispenser/Scale up 2 replicas": "init: assignByStaticWeightStrategy builds its Dispenser with init=nil (assignment.go:208)",
    "dispenser/empty clusters": "no clusters: FitError first",
    # spread.json: every select_by_region / select_best / group_clusters case scores clusters
    # with arbitrary values (20, 40, 60, 80, ...): the in-tree score plugins give only 0 or
    # 100 (cluster_locality.go:50-61), and the batch path refuses out-of-tree score plugins
    # (kp_options.n_out_of_tree_plugins), so those tables stay on the oracle
    # (tests/test_golden_spread.py) and reach the engine through the seeded universes.
}


def summary(pods):
    return {"allocatable": {"pods": str(int(pods))}, "allocated": {}, "allocating": {}}


# the bindings' resource (api.World's default apps/v1 Deployment) enabled on every
# cluster, so APIEnablement passes as the tables assume
APIS = [{"groupVersion": "apps/v1", "resources": [{"kind": "Deployment"}]}]


def cl(name, pods=None):
    c = {"name": name, "apiEnablements": APIS}
    if pods is not None:
        c["resourceSummary"] = summary(pods)
    return c


def cluster_of(detail):
    c = dict(detail.get("cluster") or {"name": detail["name"]})
    c["name"] = detail["name"]
    c["apiEnablements"] = APIS
    c["resourceSummary"] = summary(detail["alloc"])
    return c


def targets(res, names):
    return sorted((names[i], r) for i, r in res["targets"])


def engines(kind):
    if kind == "gpu":
        return Engine(0)
    return Engine(0, lib_path=os.path.join(PKG, "libkp_cpusim.so"))


_ENG = {}


def engine(kind):
    if kind not in _ENG:
        _ENG[kind] = engines(kind)
    return _ENG[kind]


def schedule(kind, clusters, binding, empty_propagation=False, plugins=api.PLUGIN_ALL):
    e = engine(kind)
    opts = api.options(empty_workload_propagation=empty_propagation, plugins=plugins)
    snap = Snapshot(e, clusters, opts)
    # the tables leave spec.resource empty (AssignReplicas never reads it); Schedule's
    # APIEnablement filter does, so the binding names the resource the clusters enable
    binding = dict(binding, apiVersion="apps/v1", kind="Deployment")
    b = Batch(snap, [binding])
    out = b.schedule()[0]
    b.close()
    snap.close()
    return out, [c["name"] for c in clusters]


KINDS = [pytest.param("cpusim", id="host"), pytest.param("gpu", id="gpu", marks=pytest.mark.gpu)]


def check(kind, name, clusters, binding, wants, want_err=False, plugins=api.PLUGIN_ALL):
    """wants: accepted target lists [(name, replicas)] (zeros included, as the
    reference function returns them)."""
    for empty in (False, True):
        got, names = schedule(kind, clusters, binding, empty, plugins)
        if want_err:
            assert got["status"] != api.STATUS_OK, f"{name}: expected an error, got {got}"
            continue
        assert got["status"] == api.STATUS_OK, f"{name} (empty propagation {empty}): {got}"
        t = targets(got, names)
        if empty:  # every selected cluster attached (attachZeroReplicasCluster)
            ok = [sorted(w + [(n, 0) for n in names if n not in dict(w)]) for w in wants]
        else:
            ok = [sorted((n, r) for n, r in w if r > 0) for w in wants]
        assert t in ok, f"{name} (empty propagation {empty}): got {t}, want one of {ok}"


def core_ids(key):
    return [c["name"] for c in CORE[key]]


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("case", CORE["distribution"], ids=core_ids("distribution"))
def test_distribution_of_replicas_engine(kind, case):
    clusters = [cluster_of(d) for d in case["clusters"]]
    want = [(t["name"], t["replicas"]) for t in case["want"]]
    check(kind, case["name"], clusters, case["binding"], [want])


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("case", CORE["assign"], ids=core_ids("assign"))
def test_assign_replicas_engine(kind, case):
    if "core/assign/" + case["name"] in NOT_EXPRESSIBLE:
        pytest.skip(NOT_EXPRESSIBLE["core/assign/" + case["name"]])
    clusters = [cluster_of(d) for d in case["clusters"]]
    # the cases score every cluster 0: ClusterLocality off (spec.Clusters would score 100;
    # the score cannot change a SEL_ALL placement, this keeps the inputs identical)
    plugins = api.PLUGIN_ALL & ~api.PLUGIN_CLUSTER_LOCALITY
    if case["wantErr"]:
        check(kind, case["name"], clusters, case["binding"], [], want_err=True, plugins=plugins)
        return
    want = [(t["name"], t["replicas"]) for t in case["want"]]
    if case["binding"]["replicas"] == 0:
        # non-workload: every candidate with 0 replicas is the reference's own answer
        # (common.go:68-80); Schedule keeps those entries with or without the flag
        got, names = schedule(kind, clusters, case["binding"], False, plugins)
        assert got["status"] == api.STATUS_OK and targets(got, names) == sorted(want)
        return
    check(kind, case["name"], clusters, case["binding"], [want], plugins=plugins)


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("case", CORE["dynamic_divide"], ids=core_ids("dynamic_divide"))
def test_dynamic_divide_engine(kind, case):
    """dynamicDivideReplicas(state) over the case's available list = a fresh binding of
    `target` replicas whose clusters' estimates are those replicas (dynamicFreshScale
    builds exactly that list, division_algorithm.go:151-172)."""
    clusters = [cl(t["name"], t["replicas"]) for t in case["available"]]
    pref = {1: "Weighted", 2: "Aggregated"}[case["strategy"]]
    rs = {"replicaSchedulingType": "Divided", "replicaDivisionPreference": pref}
    if case["strategy"] == 1:
        rs["weightPreference"] = {"dynamicWeight": "AvailableReplicas"}
    binding = {"uid": case["binding"].get("uid", ""), "replicas": case["target"], "placement": {"replicaScheduling": rs}}
    if case["wantErr"]:
        check(kind, case["name"], clusters, binding, [], want_err=True)
        return
    check(kind, case["name"], clusters, binding, [[(t["name"], t["replicas"]) for t in case["want"]]])


def webster_cases():
    return [c for c in WEB["cases"]]


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("case", webster_cases(), ids=[c["name"] for c in webster_cases()])
def test_webster_engine(kind, case):
    """AllocateWebsterSeats(newSeats, votes, nil, tie) = DynamicWeight division of a
    fresh binding of newSeats replicas over clusters whose estimates are the votes
    (SpreadReplicasByTargetClusters, util/helper/binding.go:178-183; the tie order
    is the UID's FNV parity: even -> names ascending, odd -> descending)."""
    key = "webster/" + case["name"]
    if key in NOT_EXPRESSIBLE:
        pytest.skip(NOT_EXPRESSIBLE[key])
    assert not case["init"]
    clusters = [cl(n, v) for n, v in case["votes"].items()]
    uid = UIDS["odd"] if case["tie"] == "name_desc" else UIDS["even"]
    binding = {"uid": uid, "replicas": case["newSeats"],
               "placement": {"replicaScheduling": {"replicaSchedulingType": "Divided",
                                                   "replicaDivisionPreference": "Weighted",
                                                   "weightPreference": {"dynamicWeight": "AvailableReplicas"}}}}
    want = sorted(case["expected"].items())
    if case["newSeats"] == 0:
        # 0 replicas is a non-workload binding: every candidate with 0 replicas
        # (common.go:68-80), the same as the table's all-zero answer
        got, names = schedule(kind, clusters, binding)
        assert got["status"] == api.STATUS_OK and targets(got, names) == want
        return
    check(kind, case["name"], clusters, binding, [want])


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("case", DISP["cases"], ids=[c["name"] for c in DISP["cases"]])
def test_dispenser_engine(kind, case):
    """Dispenser(num, nil, uid).AllocateByWeight(weights) = StaticWeight division with
    one clusterNames rule per weighted cluster (assignByStaticWeightStrategy,
    assignment.go:199-211)."""
    key = "dispenser/" + case["name"]
    if key in NOT_EXPRESSIBLE:
        pytest.skip(NOT_EXPRESSIBLE[key])
    assert not case["init"]
    clusters = [cl(n) for n, _ in case["weights"]]
    rules = [{"targetCluster": {"clusterNames": [n]}, "weight": w} for n, w in case["weights"]]
    binding = {"uid": UIDS[case["uid"]], "replicas": case["num"],
               "placement": {"replicaScheduling": {"replicaSchedulingType": "Divided",
                                                   "replicaDivisionPreference": "Weighted",
                                                   "weightPreference": {"staticWeightList": rules}}}}
    check(kind, case["name"], clusters, binding, [[tuple(p) for p in w] for w in case["wants"]])


def test_not_expressible_cases_exist():
    """Every listed case names a real table entry (the list stays in step with the fixtures)."""
    names = {"core/assign/" + c["name"] for c in CORE["assign"]}
    names |= {"webster/" + c["name"] for c in WEB["cases"]}
    names |= {"dispenser/" + c["name"] for c in DISP["cases"]}
    for k in NOT_EXPRESSIBLE:
        assert k in names, k
