"""Transcribes reference table-driven tests into tests/golden/*.json.

Development-container only (reads /root/reference). The produced JSON files are
committed; nothing at test or bench time reads the reference.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gotables import Call, Comp, Ref, table  # noqa: E402

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

OPS = {
    "corev1.NodeSelectorOpIn": "In", "corev1.NodeSelectorOpNotIn": "NotIn", "corev1.NodeSelectorOpExists": "Exists",
    "corev1.NodeSelectorOpDoesNotExist": "DoesNotExist", "corev1.NodeSelectorOpGt": "Gt", "corev1.NodeSelectorOpLt": "Lt",
    "metav1.LabelSelectorOpIn": "In", "metav1.LabelSelectorOpNotIn": "NotIn", "metav1.LabelSelectorOpExists": "Exists",
    "metav1.LabelSelectorOpDoesNotExist": "DoesNotExist",
    "corev1.TolerationOpExists": "Exists", "corev1.TolerationOpEqual": "Equal",
    "corev1.TaintEffectNoSchedule": "NoSchedule", "corev1.TaintEffectNoExecute": "NoExecute",
    "corev1.TaintEffectPreferNoSchedule": "PreferNoSchedule",
    "ZoneField": "zone", "RegionField": "region", "ProviderField": "provider",
    "util.ZoneField": "zone", "util.RegionField": "region", "util.ProviderField": "provider",
}


def read(path):
    with open(os.path.join(REF, path)) as f:
        return f.read()


class Ctx:
    def __init__(self, syms):
        self.syms = dict(OPS)
        self.syms.update(syms)

    def ev(self, v):
        if isinstance(v, Ref):
            if v.name in self.syms:
                return self.syms[v.name]
            raise KeyError(v.name)
        if isinstance(v, Call):
            raise ValueError("call %s" % v.fn)
        return v

    def strs(self, v):
        if v is None:
            return []
        if isinstance(v, Ref):
            return list(self.ev(v))
        return [self.ev(x) for x in v.values()]

    def strmap(self, v):
        if v is None:
            return {}
        return {self.ev(k) if not isinstance(k, str) else k: self.ev(x) for k, x in v.items}

    def reqs(self, v):
        out = []
        for e in (v.values() if v is not None else []):
            out.append({"key": self.ev(e.get("Key", "")), "operator": self.ev(e.get("Operator", "")),
                        "values": self.strs(e.get("Values"))})
        return out

    def affinity(self, a):
        if a is None:
            return None
        d = {}
        ls = a.get("LabelSelector")
        if ls is not None:
            d["labelSelector"] = {"matchLabels": self.strmap(ls.get("MatchLabels")),
                                  "matchExpressions": self.reqs(ls.get("MatchExpressions"))}
        fs = a.get("FieldSelector")
        if fs is not None:
            d["fieldSelector"] = {"matchExpressions": self.reqs(fs.get("MatchExpressions"))}
        d["clusterNames"] = self.strs(a.get("ClusterNames"))
        d["exclude"] = self.strs(a.get("ExcludeClusters"))
        return d


def selector_tests():
    src = read("pkg/util/selector_test.go")
    rows, line = table(src, "TestClusterMatches")
    cluster = {"name": "cluster1", "labels": {"foo": "bar"}, "zones": ["zone1", "zone2", "zone3"],
               "region": "region1", "provider": "provider1"}
    ctx = Ctx({"cluster.Name": "cluster1", "cluster.Spec.Zones": cluster["zones"],
               "cluster.Spec.Region": "region1", "cluster.Spec.Provider": "provider1"})
    cases = []
    for r in rows:
        cases.append({"name": r.get("name"), "affinity": ctx.affinity(r.get("affinity")), "want": r.get("want")})
    zrows, zline = table(src, "Test_matchZones")
    zcases = []
    for r in zrows:
        e = r.get("zoneMatchExpression")
        zcases.append({"name": r.get("name"), "expr": ctx.reqs(Comp(None, [(None, e)]))[0],
                       "zones": ctx.strs(r.get("zones")), "want": r.get("matched")})
    return {"source": "pkg/util/selector_test.go:%d (TestClusterMatches), :%d (Test_matchZones)" % (line, zline),
            "note": "ClusterMatches over the test's fixed cluster; matchZones through a FieldSelector holding only the zone expression on a cluster with the given zones.",
            "cluster": cluster, "cases": cases, "zoneCases": zcases}


def main():
    out = {"selector.json": selector_tests()}
    for name, data in out.items():
        with open(os.path.join(OUT, name), "w") as f:
            json.dump(data, f, indent=1)
        print(name, len(data.get("cases", [])))


if __name__ == "__main__":
    main()
