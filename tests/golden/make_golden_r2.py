"""Transcribes more of the reference's table-driven tests into tests/golden/*.json
(round 2: filter/score plugins, spread selection, core assignment, the FF
simulator). Development-container only (reads /root/reference); the JSON it
writes is committed and is all the test suite reads.

    python tests/golden/make_golden_r2.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from goconv import Conv  # noqa: E402
from gotables import Call, Comp, Parser, Ref, func_body, table, tokenize  # noqa: E402

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def read(path):
    with open(os.path.join(REF, path), encoding="utf-8") as f:
        return f.read()


def code_fit(code):
    return {"Success": True, "Unschedulable": False, "Error": False}[code]


def plugin_filter_cases(path, func, plugin):
    rows, line = table(read(path), func)
    cv = Conv()
    cases = []
    for r in rows:
        cases.append({"name": r.get("name"), "plugin": plugin,
                      "binding": cv.spec(r.get("bindingSpec"), r.get("bindingStatus")),
                      "cluster": cv.cluster(r.get("cluster") or Comp(None, [])),
                      "fit": code_fit(cv.ev(r.get("expectedCode")))})
    return cases, "%s:%d (%s)" % (path, line, func)


def plugins():
    P = "pkg/scheduler/framework/plugins/"
    out, src = [], []
    for path, func, plugin in [
        (P + "tainttoleration/taint_toleration_test.go", "TestTaintToleration_Filter", "TaintToleration"),
        (P + "apienablement/api_enablement_test.go", "TestAPIEnablement_Filter", "APIEnablement"),
        (P + "clusteraffinity/cluster_affinity_test.go", "TestClusterAffinity_Filter", "ClusterAffinity"),
        (P + "spreadconstraint/spread_constraint_test.go", "TestSpreadConstraint_Filter", "SpreadConstraint"),
        (P + "clustereviction/cluster_eviction_test.go", "TestClusterEviction_Filter", "ClusterEviction"),
    ]:
        c, s = plugin_filter_cases(path, func, plugin)
        out += c
        src.append(s)
    # ClusterLocality.Score
    path = P + "clusterlocality/cluster_locality_test.go"
    rows, line = table(read(path), "TestClusterLocality_Score")
    cv = Conv()
    scores = [{"name": r.get("name"), "plugin": "ClusterLocality", "binding": cv.spec(r.get("bindingSpec")),
               "cluster": cv.cluster(r.get("cluster") or Comp(None, [])), "score": cv.ev(r.get("expectedScore"))}
              for r in rows]
    src.append("%s:%d (TestClusterLocality_Score)" % (path, line))
    # Cluster.APIEnablement (pkg/apis/cluster/v1alpha1/cluster_helper.go:46-67), as the filter sees it
    path = "pkg/apis/cluster/v1alpha1/cluster_helper_test.go"
    rows, line = table(read(path), "TestAPIEnablement")
    cv = Conv({"APIEnabled": "APIEnabled", "APIDisabled": "APIDisabled", "APIUnknown": "APIUnknown"})
    for r in rows:
        g = r.get("gvk")
        grp, ver, kind = cv.ev(g.get("Group", "")), cv.ev(g.get("Version", "")), cv.ev(g.get("Kind", ""))
        b = {"apiVersion": grp + "/" + ver if grp else ver, "kind": kind, "placement": {}}
        out.append({"name": "cluster_helper: " + r.get("name"), "plugin": "APIEnablement", "binding": b,
                    "cluster": cv.cluster(r.get("cluster")), "fit": cv.ev(r.get("expected")) == "APIEnabled"})
    src.append("%s:%d (TestAPIEnablement; APIDisabled and APIUnknown both fail the filter, "
               "api_enablement.go:51-78)" % (path, line))
    return {"source": src, "filters": out, "scores": scores}


def func_literal(src, func):
    """The composite literal a helper function returns (`return T{...}`), and its line."""
    body, line = func_body(src, func)
    i = body.index("return ")
    return Parser(tokenize(body[i + len("return "):])).parse_value(), line


def strip_funcs(src, key):
    """Replaces `key: func(...) ... { ... }` literals by `key: true` (the parser reads no code)."""
    out, i = [], 0
    while True:
        j = src.find(key + ": func(", i)
        if j < 0:
            out.append(src[i:])
            return "".join(out)
        k = src.index("{", src.index(")", j))  # the body opens after the parameter list
        depth = 0
        while True:
            if src[k] == "{":
                depth += 1
            elif src[k] == "}":
                depth -= 1
                if depth == 0:
                    break
            k += 1
        out.append(src[i:j] + key + ": true")
        i = k + 1


def detail(cv, c):
    """ClusterDetailInfo literal -> {name, score, avail, ovf, cluster (topology dict or None)}."""
    cl = c.get("Cluster")
    return {"name": cv.ev(c.get("Name", "")), "score": cv.ev(c.get("Score", 0)),
            "avail": cv.ev(c.get("AvailableReplicas", 0)), "ovf": cv.ev(c.get("OverflowOrder", 0)),
            "cluster": cv.cluster(cl) if cl is not None else None}


def topo(name, provider, region, zone):  # NewClusterWithTopology (select_clusters_test.go:31-40)
    return {"name": name, "provider": provider, "region": region, "zones": [zone]}


def spread():
    SP = "pkg/scheduler/core/spreadconstraint/"
    cv = Conv({"NewClusterWithTopology": topo})
    res = {"source": []}
    # selectGroups
    rows, line = table(read(SP + "select_groups_test.go"), "TestSelectGroups")
    res["select_groups"] = [{"name": r.get("name"),
                             "groups": [{"name": cv.ev(g.get("name")), "value": cv.ev(g.get("value")),
                                         "weight": cv.ev(g.get("weight"))}
                                        for g in (r.get("groups").values() if r.get("groups") is not None else [])],
                             "min": r.get("minConstraints"), "max": r.get("maxConstraints"), "target": r.get("target"),
                             "expected": cv.strs(r.get("expected"))} for r in rows]
    res["source"].append(SP + "select_groups_test.go:%d (TestSelectGroups)" % line)
    # selectBestClustersByRegion
    rows, line = table(read(SP + "select_clusters_by_region_test.go"), "Test_selectBestClustersByRegion")
    cases = []
    for r in rows:
        a = r.get("args")
        scm = {cv.key(k): (cv.ev(v.get("MinGroups", 0)), cv.ev(v.get("MaxGroups", 0)))
               for k, v in a.get("spreadConstraintMap").items}
        regions = []
        for k, v in a.get("groupClustersInfo").get("Regions").items:
            regions.append({"name": cv.ev(v.get("Name", k)), "score": cv.ev(v.get("Score", 0)),
                            "clusters": [detail(cv, c) for c in (v.get("Clusters").values()
                                                                  if v.get("Clusters") is not None else [])]})
        want = [cv.cluster(c)["name"] for c in (r.get("want").values() if r.get("want") is not None else [])]
        cases.append({"name": r.get("name"), "region": scm.get("region", (0, 0)), "cluster": scm.get("cluster", (0, 0)),
                      "regions": regions, "want": want, "wantErr": bool(r.get("wantErr"))})
    res["select_by_region"] = cases
    res["source"].append(SP + "select_clusters_by_region_test.go:%d (Test_selectBestClustersByRegion)" % line)
    # SelectBestClusters over generateClusterInfo()
    import re
    src = read(SP + "select_clusters_test.go")
    lit, _ = func_literal(src, "generateClusterInfo")
    infos = [detail(cv, c) for c in lit.values()]
    src = re.sub(r"clusterInfos\[(\d+)\]", r"CI(\1)", src)
    cv2 = Conv({"NewClusterWithTopology": topo, "clusterInfos": infos, "CI": lambda i: infos[i]})
    rows, line = table(src, "TestSelectBestClusters")
    cases = []
    for r in rows:
        a = r.get("args")
        want = r.get("want")
        cases.append({"name": r.get("name"), "binding": {"placement": cv2.placement(a.get("placement")),
                                                         "replicas": 0},
                      "clusters": cv2.ev(a.get("groupClustersInfo").get("Clusters")),
                      "need": cv2.ev(a.get("needReplicas")),
                      "want": [cv2.ev(w)["name"] for w in want.values()] if want is not None else None,
                      "wantErr": r.get("wantErr") is not None})
    res["select_best"] = cases
    res["source"].append(SP + "select_clusters_test.go:%d (TestSelectBestClusters)" % line)
    # GroupClustersWithScore over generateClusterScore(), calAvailableReplicasFunc = 100
    src = read(SP + "group_clusters_test.go")
    lit, _ = func_literal(src, "generateClusterScore")
    scored = [{"cluster": cv.cluster(c.get("Cluster")), "score": cv.ev(c.get("Score"))} for c in lit.values()]
    rows, line = table(src, "Test_GroupClustersWithScore")
    cases = []
    for r in rows:
        a, w = r.get("args"), r.get("want")
        cases.append({"name": r.get("name"), "clusters": scored, "avail": 100,
                      "binding": {"placement": cv.placement(a.get("placement")), "replicas": 0},
                      "order": cv.strs(w.get("clusters")), "zones": w.get("zoneCnt", 0),
                      "regions": w.get("regionCnt", 0), "providers": w.get("providerCnt", 0)})
    res["group_clusters"] = cases
    res["source"].append(SP + "group_clusters_test.go:%d (Test_GroupClustersWithScore)" % line)
    # calcGroupScore: generateArgs() with generateClusterScores / generateRbSpec
    def gen_scores(n, scores, reps):
        scores, reps = [cv.ev(x) for x in scores.values()], [cv.ev(x) for x in reps.values()]
        return [{"name": "member%d" % (i + 1), "score": scores[i], "avail": reps[i], "ovf": 0, "cluster": None}
                for i in range(n)]

    def rbspec(rep, kind):
        rs = {"duplicated": {"replicaSchedulingType": "Duplicated"},
              "aggregated": {"replicaSchedulingType": "Divided", "replicaDivisionPreference": "Aggregated"},
              "dynamicWeight": {"replicaSchedulingType": "Divided", "replicaDivisionPreference": "Weighted",
                                "weightPreference": {"dynamicWeight": "AvailableReplicas"}},
              "staticWeight": {"replicaSchedulingType": "Divided", "replicaDivisionPreference": "Weighted",
                               "weightPreference": {"staticWeightList": []}}}[kind]
        return {"replicas": rep, "placement": {"replicaScheduling": rs}}
    src2 = re.sub(r"generateRbSpec\((\d+)\)\[(\w+)\]", r'RB(\1, "\2")', src)
    cv3 = Conv({"generateClusterScores": gen_scores, "RB": rbspec})
    rows, line = table(src2, "generateArgs", var="argsList")
    cases = []
    for r in rows:
        cases.append({"name": "id %d" % r.get("id"), "a": cv3.ev(Call("generateClusterScores", r.get("clusters1").args))
                      if isinstance(r.get("clusters1"), Call) else None,
                      "b": cv3.ev(r.get("clusters2")), "binding": cv3.ev(r.get("rbSpec")),
                      "minGroups": r.get("minGroups", 0), "aWins": r.get("group1Wins")})
    for c in cases:
        if c["a"] is None:
            raise ValueError(c)
    res["calc_group_score"] = cases
    res["source"].append(SP + "group_clusters_test.go:%d (Test_CalcGroupScore via generateArgs)" % line)
    rows, line = table(src, "Test_CalcGroupScoreForDuplicate")
    res["calc_group_score_dup"] = [{"name": r.get("name"),
                                    "clusters": [detail(cv, c) for c in r.get("clusters").values()],
                                    "binding": {"replicas": cv.ev(r.get("rbSpec").get("Replicas", 0)),
                                                "placement": {"replicaScheduling": {"replicaSchedulingType":
                                                                                    "Duplicated"}}},
                                    "score": r.get("watScore")} for r in rows]
    res["source"].append(SP + "group_clusters_test.go:%d (Test_CalcGroupScoreForDuplicate: calcGroupScore"
                         " dispatches Duplicated bindings to it, group_clusters.go:238-241)" % line)
    # sortClusters
    src = strip_funcs(read(SP + "util_test.go"), "compareFunction")
    rows, line = table(src, "Test_sortClusters")
    res["sort_clusters"] = [{"name": r.get("name"), "infos": [detail(cv, c) for c in r.get("infos").values()],
                             "want": [cv.ev(c.get("Name")) for c in r.get("want").values()],
                             "withAvail": bool(r.get("compareFunction"))} for r in rows]
    res["source"].append(SP + "util_test.go:%d (Test_sortClusters)" % line)
    return res


def new_cluster(name):  # helper.NewCluster (test/helper/resource.go:680-687)
    return {"name": name}


def detail2(cv, c):
    """ClusterDetailInfo with every field the assignment reads."""
    cl = c.get("Cluster")
    return {"name": cv.ev(c.get("Name", "")), "score": cv.ev(c.get("Score", 0)),
            "avail": cv.ev(c.get("AvailableReplicas", 0)), "alloc": cv.ev(c.get("AllocatableReplicas", 0)),
            "ovf": cv.ev(c.get("OverflowOrder", 0)), "cluster": cv.cluster(cl) if cl is not None else None}


def core():
    CORE = "pkg/scheduler/core/"
    cv = Conv({"helper.NewCluster": new_cluster})
    res = {"source": []}
    # Test_DistributionOfReplicas: genericScheduler.assignReplicas over ClusterDetailInfo lists
    rows, line = table(read(CORE + "generic_scheduler_test.go"), "Test_DistributionOfReplicas")
    res["distribution"] = [{"name": r.get("name"), "clusters": [detail2(cv, c) for c in r.get("clusters").values()],
                            "binding": cv.spec(r.get("object")), "want": cv.targets(r.get("result"))} for r in rows]
    res["source"].append(CORE + "generic_scheduler_test.go:%d (Test_DistributionOfReplicas)" % line)
    # TestAssignReplicas
    rows, line = table(read(CORE + "common_test.go"), "TestAssignReplicas")
    res["assign"] = [{"name": r.get("name"), "clusters": [detail2(cv, c) for c in r.get("clusters").values()],
                      "binding": cv.spec(r.get("spec"), r.get("status")),
                      "want": cv.targets(r.get("expectedResult")) if r.get("expectedResult") is not None else None,
                      "wantErr": bool(r.get("expectedError"))} for r in rows]
    res["source"].append(CORE + "common_test.go:%d (TestAssignReplicas)" % line)
    # TestSelectClusters: SelectClusters over scored clusters; no cluster has a ResourceSummary
    # and no spec has replicas, so calAvailableReplicas answers 0 for every cluster
    rows, line = table(read(CORE + "common_test.go"), "TestSelectClusters")
    cases = []
    for r in rows:
        b = cv.spec(r.get("spec"), r.get("status"))
        b["placement"] = cv.placement(r.get("placement"))
        cases.append({"name": r.get("name"), "binding": b,
                      "clusters": [cv.cluster(x.get("Cluster")) for x in r.get("clustersScore").values()],
                      "scores": [cv.ev(x.get("Score", 0)) for x in r.get("clustersScore").values()],
                      "want": sorted(cv.cluster(x)["name"] for x in (r.get("expectedResult").values()
                                                                     if r.get("expectedResult") else [])),
                      "wantErr": bool(r.get("expectedError"))})
    res["select"] = cases
    res["source"].append(CORE + "common_test.go:%d (TestSelectClusters)" % line)
    # Test_dynamicDivideReplicas
    cv2 = Conv({"DynamicWeightStrategy": 1, "AggregatedStrategy": 2, "StaticWeightStrategy": 3,
                "DuplicatedStrategy": 4})
    rows, line = table(read(CORE + "division_algorithm_test.go"), "Test_dynamicDivideReplicas")
    cases = []
    for r in rows:
        st = r.get("state")
        cases.append({"name": r.get("name"), "available": cv2.targets(st.get("availableClusters")),
                      "target": cv2.ev(st.get("targetReplicas", 0)),
                      "availableReplicas": cv2.ev(st.get("availableReplicas", 0)),
                      "strategy": cv2.ev(st.get("strategyType")), "binding": cv2.spec(st.get("spec")),
                      "want": cv2.targets(r.get("want")), "wantErr": bool(r.get("wantErr"))})
    res["dynamic_divide"] = cases
    res["source"].append(CORE + "division_algorithm_test.go:%d (Test_dynamicDivideReplicas)" % line)
    return res


def sets():
    """GeneralEstimator component-set tables (estimator/client/general_test.go) and the
    FF simulator table (estimator/scheduling_simulator_components_test.go)."""
    res = {"source": []}
    GEN = "pkg/estimator/client/general_test.go"
    src = read(GEN)
    cv = Conv({"GPU": "nvidia.com/gpu", "BIGU": 100, "q": lambda x: x})

    def comp(name, replicas, rl):  # general_test.go:251-259
        return {"name": cv.ev(name), "replicas": cv.ev(replicas),
                "replicaRequirements": {"resourceRequest": cv.qmap(rl)}}
    cv.syms["comp"] = comp
    rows, line = table(src, "TestGetMaximumSetsBasedOnResourceModels")
    res["models"] = [{"name": r.get("name"), "cluster": cv.cluster(r.get("cluster")),
                      "components": cv.components(r.get("components")), "upperBound": cv.ev(r.get("upperBound")),
                      "expectError": bool(cv.ev(r.get("expectError", False))),
                      "expectedSets": cv.ev(r.get("expectedSets"))} for r in rows]
    res["source"].append(GEN + ":%d (TestGetMaximumSetsBasedOnResourceModels)" % line)
    rows, line = table(src, "TestGetMaxAvailableComponentSetsGeneral")
    res["general"] = [{"name": r.get("name"), "cluster": cv.cluster(r.get("cluster") or Comp(None, [])),
                       "components": cv.components(r.get("components")), "expected": cv.ev(r.get("expected"))}
                      for r in rows]
    res["source"].append(GEN + ":%d (TestGetMaxAvailableComponentSetsGeneral)" % line)
    SIM = "pkg/estimator/scheduling_simulator_components_test.go"
    ssrc = read(SIM).replace("(&pb.ComponentReplicaRequirements{}).MustSetResourceRequest(", "RR(")
    cs = Conv({"RR": lambda rl: cs.qmap(rl), "createNodeInfo": lambda name, rl: {"name": name, "allocatable": rl}})
    rows, line = table(ssrc, "TestSchedulingSimulator_SimulateSchedulingFF")
    ff = []
    for r in rows:
        nodes = [{"name": cs.ev(n.args[0]), "allocatable": cs.qmap(n.args[1])} for n in r.get("nodes").values()]
        comps = []
        for c in r.get("components").values():
            rr = c.get("ReplicaRequirements")
            d = {"name": cs.ev(c.get("Name", "")), "replicas": cs.ev(c.get("Replicas", 0))}
            if rr is not None:
                d["replicaRequirements"] = {"resourceRequest": cs.qmap(rr.args[0]) if isinstance(rr, Call) else {}}
            comps.append(d)
        ff.append({"name": r.get("name"), "nodes": nodes, "components": comps,
                   "upperBound": cs.ev(r.get("upperBound")), "expectedSets": cs.ev(r.get("expectedSets"))})
    res["ff"] = ff
    res["source"].append(SIM + ":%d (TestSchedulingSimulator_SimulateSchedulingFF)" % line)
    return res


def main():
    outs = {"plugins.json": plugins(), "spread.json": spread(), "core.json": core(), "sets.json": sets()}
    for name, data in outs.items():
        with open(os.path.join(OUT, name), "w") as f:
            json.dump(data, f, indent=1)
        print(name, {k: len(v) for k, v in data.items() if isinstance(v, list)})


if __name__ == "__main__":
    main()
