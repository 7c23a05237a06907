"""Transcribes the estimator server's node tables into tests/golden/nodes_server.json.

Sources (read as text; the vectors below are the tables' data, restated in the
engine's dict form — a node is {name, labels, taints, allocatable, requested, pods},
`requested` the sum of its pods' requests and `pods` their count, as the
estimator's NodeInfo holds them):

- pkg/estimator/server/server_test.go:43-230
  TestAccurateSchedulerEstimatorServer_MaxAvailableReplicas (5 cases); nodes from
  test/helper/resource.go:561-672 (NewNode / MakeNodeWithLabels / MakeNodeWithTaints:
  milli-cpu, BinarySI memory and storage, DecimalSI pods), pods from
  NewPodWithRequest (:537-558); units ResourceUnitCPU = 1000 milli, Mem = 1Gi (:47-54).
- pkg/estimator/scheduling_simulator_components_test.go:32-144 TestMatchNode: cases
  2-4 (case 1 is a NodeInfo without a Node object, which kp_node cannot express).
  MatchNode is observed through kp_node_max_replicas on the single node: the
  reference node has no pods allocatable (MaxDivided would be 0 either way), so
  the fixture adds "pods": "110" and expects a positive answer exactly when the
  reference expects a match.
- pkg/estimator/server/framework/plugins/noderesource/noderesource_test.go:32-468
  TestNodeResourceEstimator_EstimateComponents: 13 of 14 cases ("plugin disabled"
  is the plugin's own switch, outside the estimate); makeNode / makePod (:489-529).

Run: python tests/golden/make_golden_nodes.py  (writes nodes_server.json next to it)
"""
import json
import os

GI = 1024 ** 3


def node(name, cpu_milli, mem, pods, storage, labels=None, taints=None, pod_reqs=()):
    d = {"name": name, "allocatable": {"cpu": f"{cpu_milli}m", "memory": str(mem), "pods": str(pods),
                                       "ephemeral-storage": str(storage)}}
    if labels:
        d["labels"] = labels
    if taints:
        d["taints"] = taints
    if pod_reqs:
        c = sum(p[0] for p in pod_reqs)
        m = sum(p[1] for p in pod_reqs)
        e = sum(p[2] for p in pod_reqs)
        d["requested"] = {"cpu": f"{c}m", "memory": str(m), "ephemeral-storage": str(e)}
        d["pods"] = len(pod_reqs)
    return d


def server_nodes(pods1=11, pods2=11, labels1=None, labels2=None, taints1=None, taints2=None):
    # node 1 pods: (1 cpu, 3Gi), (3 cpu, 3Gi), (2 cpu, 4Gi, 2Gi storage); node 2: (4, 8Gi, 2Gi), (1, 3Gi, 2Gi)
    p1 = [(1000, 3 * GI, 0), (3000, 3 * GI, 0), (2000, 4 * GI, 2 * GI)]
    p2 = [(4000, 8 * GI, 2 * GI), (1000, 3 * GI, 2 * GI)]
    return [node("machine1", 8000, 16 * GI, pods1, 16 * GI, labels1, taints1, p1),
            node("machine2", 8000, 16 * GI, pods2, 16 * GI, labels2, taints2, p2),
            node("machine3", 8000, 16 * GI, 11, 16 * GI)]


REQ = {"cpu": "1000m", "memory": str(2 * GI), "ephemeral-storage": "0"}

server = [
    {"name": "normal", "nodes": server_nodes(), "request": REQ, "want": 12},
    {"name": "pod resource strict", "nodes": server_nodes(pods1=4, pods2=3), "request": REQ, "want": 10},
    {"name": "request with node selector", "nodes": server_nodes(labels1={"a": "1"}, labels2={"a": "3", "b": "2"}),
     "request": REQ, "claim": {"nodeSelector": {"a": "3"}}, "want": 2},
    {"name": "request with node affinity", "nodes": server_nodes(labels1={"a": "1"}, labels2={"a": "3", "b": "2"}),
     "request": REQ, "claim": {"nodeAffinity": {"nodeSelectorTerms": [
         {"matchExpressions": [{"key": "a", "operator": "Gt", "values": ["0"]}]}]}}, "want": 4},
    {"name": "request with tolerations",
     "nodes": server_nodes(taints1=[{"key": "key1", "value": "value1", "effect": "NoSchedule"}],
                           taints2=[{"key": "key2", "value": "value2", "effect": "NoSchedule"}]),
     "request": REQ, "claim": {"tolerations": [{"key": "key1", "operator": "Equal", "value": "value1"}]}, "want": 10},
]

ZONE_WEST = {"nodeAffinity": {"nodeSelectorTerms": [
    {"matchExpressions": [{"key": "zone", "operator": "In", "values": ["us-west"]}]}]}}
match_node = [
    {"name": "no constraints - should match", "node_labels": {}, "claim": None, "match": True},
    {"name": "node affinity matches", "node_labels": {"zone": "us-west"}, "claim": ZONE_WEST, "match": True},
    {"name": "node affinity does not match", "node_labels": {"zone": "us-east"}, "claim": ZONE_WEST, "match": False},
]
for c in match_node:
    c["nodes"] = [{"name": "node1", "labels": c.pop("node_labels"), "allocatable": {"cpu": "4", "pods": "110"}}]
    c["request"] = {"cpu": "1"}


def mnode(name, cpu, mem, pods="10", labels=None, req=None, npods=0):
    d = {"name": name, "labels": labels or {}, "allocatable": {"cpu": cpu, "memory": mem, "pods": pods}}
    if req:
        d["requested"] = req
        d["pods"] = npods
    return d


def comp(cpu, mem, replicas, claim=None):
    rr = {"resourceRequest": {"cpu": cpu, "memory": mem}}
    if claim is not None:
        rr["nodeClaim"] = claim
    return {"replicas": replicas, "replicaRequirements": rr}


def zone(v):
    return {"nodeAffinity": {"nodeSelectorTerms": [{"matchExpressions": [{"key": "zone", "operator": "In",
                                                                         "values": [v]}]}]}}


INT32_MAX = 2147483647
two_zone = [mnode("node1", "4", "8Gi", labels={"zone": "us-west"}), mnode("node2", "4", "8Gi", labels={"zone": "us-east"})]
components = [
    {"name": "single component single replica fits in single node", "nodes": [mnode("node1", "4", "8Gi")],
     "components": [comp("1", "1Gi", 1)], "want": 4},
    {"name": "single component multiple replicas fits in single node", "nodes": [mnode("node1", "4", "8Gi")],
     "components": [comp("1", "1Gi", 2)], "want": 2},
    {"name": "multiple components fit in single node", "nodes": [mnode("node1", "10", "10Gi")],
     "components": [comp("2", "2Gi", 1), comp("3", "3Gi", 1)], "want": 2},
    {"name": "components spread across multiple nodes", "nodes": [mnode("node1", "6", "6Gi"), mnode("node2", "6", "6Gi")],
     "components": [comp("3", "3Gi", 2), comp("2", "2Gi", 1)], "want": 1},
    {"name": "insufficient resources", "nodes": [mnode("node1", "2", "2Gi")],
     "components": [comp("3", "3Gi", 1)], "want": 0},
    {"name": "node with existing pods", "nodes": [mnode("node1", "4", "8Gi", req={"cpu": "1", "memory": "2Gi"}, npods=1)],
     "components": [comp("1", "2Gi", 1)], "want": 3},
    {"name": "node affinity constraints", "nodes": two_zone, "components": [comp("1", "1Gi", 1, zone("us-west"))],
     "want": 4},
    {"name": "no component match node affinity constraints", "nodes": two_zone,
     "components": [comp("1", "1Gi", 4, zone("us-south"))], "want": 0},
    {"name": "empty components", "nodes": [mnode("node1", "4", "8Gi")], "components": [], "want": INT32_MAX},
    {"name": "assumed workload reduces available capacity", "nodes": [mnode("node1", "4", "8Gi")],
     "components": [comp("1", "1Gi", 1)], "assumed": [{"components": [comp("1", "1Gi", 1)]}], "want": 3},
    {"name": "multiple assumed workloads reduce capacity", "nodes": [mnode("node1", "6", "6Gi")],
     "components": [comp("1", "1Gi", 1)],
     "assumed": [{"components": [comp("1", "1Gi", 1)]}, {"components": [comp("2", "2Gi", 1)]}], "want": 3},
    {"name": "assumed workload cannot be placed - deduction skipped, capacity unchanged",
     "nodes": [mnode("node1", "4", "4Gi")], "components": [comp("1", "1Gi", 1)],
     "assumed": [{"components": [comp("100", "100Gi", 1)]}], "want": 4},
    {"name": "assumed workload with empty components is ignored", "nodes": [mnode("node1", "4", "4Gi")],
     "components": [comp("1", "1Gi", 1)], "assumed": [{"components": []}], "want": 4},
]

out = {"server": server, "match_node": match_node, "components": components}
with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "nodes_server.json"), "w") as f:
    json.dump(out, f, indent=1)
