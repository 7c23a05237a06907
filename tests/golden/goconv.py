"""Converts parsed Go composite literals of Karmada API types (gotables.Comp) into
the dict layout of karmada_amd/api.py (the JSON field names of the reference
types), for transcribing reference tests into tests/golden/*.json.

Development-container only: make_golden_r2.py drives it over /root/reference.
"""
from gotables import Call, Comp, Ref

CONST = {
    # policyv1alpha1
    "policyv1alpha1.SpreadByFieldCluster": "cluster", "policyv1alpha1.SpreadByFieldRegion": "region",
    "policyv1alpha1.SpreadByFieldZone": "zone", "policyv1alpha1.SpreadByFieldProvider": "provider",
    "policyv1alpha1.ReplicaSchedulingTypeDuplicated": "Duplicated",
    "policyv1alpha1.ReplicaSchedulingTypeDivided": "Divided",
    "policyv1alpha1.ReplicaDivisionPreferenceAggregated": "Aggregated",
    "policyv1alpha1.ReplicaDivisionPreferenceWeighted": "Weighted",
    "policyv1alpha1.DynamicWeightByAvailableReplicas": "AvailableReplicas",
    # corev1
    "corev1.TolerationOpExists": "Exists", "corev1.TolerationOpEqual": "Equal",
    "corev1.TaintEffectNoSchedule": "NoSchedule", "corev1.TaintEffectNoExecute": "NoExecute",
    "corev1.TaintEffectPreferNoSchedule": "PreferNoSchedule",
    "corev1.ResourceCPU": "cpu", "corev1.ResourceMemory": "memory", "corev1.ResourcePods": "pods",
    "corev1.ResourceEphemeralStorage": "ephemeral-storage",
    "uint": lambda x: x,
    "corev1.NodeSelectorOpIn": "In", "corev1.NodeSelectorOpNotIn": "NotIn",
    "corev1.NodeSelectorOpExists": "Exists", "corev1.NodeSelectorOpDoesNotExist": "DoesNotExist",
    "corev1.NodeSelectorOpGt": "Gt", "corev1.NodeSelectorOpLt": "Lt",
    "metav1.LabelSelectorOpIn": "In", "metav1.LabelSelectorOpNotIn": "NotIn",
    "metav1.LabelSelectorOpExists": "Exists", "metav1.LabelSelectorOpDoesNotExist": "DoesNotExist",
    # framework
    "framework.Success": "Success", "framework.Unschedulable": "Unschedulable", "framework.Error": "Error",
    "framework.MaxClusterScore": 100, "framework.MinClusterScore": 0,
    "ClusterMember1": "member1", "ClusterMember2": "member2", "ClusterMember3": "member3",
    "ClusterMember4": "member4",
}


class Conv:
    def __init__(self, syms=None):
        self.syms = dict(CONST)
        self.syms.update(syms or {})

    # -- scalars ---------------------------------------------------------------------
    def ev(self, v):
        if isinstance(v, Ref):
            if v.name in self.syms:
                return self.syms[v.name]
            raise KeyError(v.name)
        if isinstance(v, Call):
            if v.fn in ("resource.MustParse", "MustParse") and len(v.args) == 1:
                return self.ev(v.args[0])
            if v.fn.endswith("NewQuantity") or v.fn.endswith("NewMilliQuantity"):
                raise ValueError("quantity call %s" % v.fn)
            if v.fn in self.syms and callable(self.syms[v.fn]):
                return self.syms[v.fn](*[self.ev(a) for a in v.args])
            if v.fn in ("int32", "int64", "int", "string", "ptr.To", "pointer.Int32", "new"):
                return self.ev(v.args[0])
            raise ValueError("call %s" % v.fn)
        if isinstance(v, Comp) and v.typ is None:
            return v
        return v

    def key(self, k):
        """A map-literal key: the parser gives identifiers as their names (constants resolved)."""
        if isinstance(k, str):
            return self.syms.get(k, k)
        return self.ev(k)

    def strs(self, v):
        if v is None:
            return []
        if isinstance(v, (Ref, Call)):
            return list(self.ev(v))
        return [self.ev(x) for x in v.values()]

    def strmap(self, v):
        if v is None:
            return {}
        return {self.key(k): self.ev(x) for k, x in v.items}

    def qmap(self, v):
        """corev1.ResourceList -> {name: quantity string}."""
        if v is None:
            return {}
        out = {}
        for k, x in v.items:
            name = self.key(k)
            q = self.ev(x)
            out[name] = str(q)
        return out

    # -- policy ------------------------------------------------------------------------
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

    def tolerations(self, v):
        out = []
        for t in (v.values() if v is not None else []):
            out.append({"key": self.ev(t.get("Key", "")), "operator": self.ev(t.get("Operator", "")),
                        "value": self.ev(t.get("Value", "")), "effect": self.ev(t.get("Effect", ""))})
        return out

    def placement(self, p):
        if p is None:
            return None
        d = {}
        if p.get("ClusterAffinity") is not None:
            d["clusterAffinity"] = self.affinity(p.get("ClusterAffinity"))
        terms = []
        for t in (p.get("ClusterAffinities").values() if p.get("ClusterAffinities") is not None else []):
            a = self.affinity(t.get("ClusterAffinity")) or {}
            a["affinityName"] = self.ev(t.get("AffinityName", ""))
            a["overflowAffinities"] = [self.affinity(o.get("ClusterAffinity")) for o in
                                       (t.get("OverflowAffinities").values() if t.get("OverflowAffinities") else [])]
            terms.append(a)
        if terms:
            d["clusterAffinities"] = terms
        d["clusterTolerations"] = self.tolerations(p.get("ClusterTolerations"))
        sc = []
        for s in (p.get("SpreadConstraints").values() if p.get("SpreadConstraints") is not None else []):
            sc.append({"spreadByField": self.ev(s.get("SpreadByField", "")),
                       "spreadByLabel": self.ev(s.get("SpreadByLabel", "")),
                       "maxGroups": self.ev(s.get("MaxGroups", 0)), "minGroups": self.ev(s.get("MinGroups", 0))})
        d["spreadConstraints"] = sc
        rs = p.get("ReplicaScheduling")
        if rs is not None:
            r = {"replicaSchedulingType": self.ev(rs.get("ReplicaSchedulingType", "")),
                 "replicaDivisionPreference": self.ev(rs.get("ReplicaDivisionPreference", ""))}
            wp = rs.get("WeightPreference")
            if wp is not None:
                r["weightPreference"] = {
                    "staticWeightList": [{"targetCluster": self.affinity(w.get("TargetCluster")) or {},
                                          "weight": self.ev(w.get("Weight", 0))}
                                         for w in (wp.get("StaticWeightList").values()
                                                   if wp.get("StaticWeightList") is not None else [])],
                    "dynamicWeight": self.ev(wp.get("DynamicWeight", ""))}
            d["replicaScheduling"] = r
        return d

    # -- binding -------------------------------------------------------------------------
    def targets(self, v):
        return [{"name": self.ev(t.get("Name", "")), "replicas": self.ev(t.get("Replicas", 0))}
                for t in (v.values() if v is not None else [])]

    def spec(self, s, status=None):
        """workv1alpha2.ResourceBindingSpec (+ Status) -> binding dict."""
        d = {"uid": "", "apiVersion": "", "kind": "", "name": "", "namespace": ""}
        if s is None:
            s = Comp(None, [])
        r = s.get("Resource")
        if r is not None:
            d.update(uid=self.ev(r.get("UID", "")), apiVersion=self.ev(r.get("APIVersion", "")),
                     kind=self.ev(r.get("Kind", "")), name=self.ev(r.get("Name", "")),
                     namespace=self.ev(r.get("Namespace", "")))
        d["replicas"] = self.ev(s.get("Replicas", 0))
        rr = s.get("ReplicaRequirements")
        if rr is not None:
            d["replicaRequirements"] = {"resourceRequest": self.qmap(rr.get("ResourceRequest"))}
            if rr.get("NodeClaim") is not None:
                d["replicaRequirements"]["nodeClaim"] = {}
        comps = s.get("Components")
        if comps is not None:
            d["components"] = len(comps.values())
        d["clusters"] = self.targets(s.get("Clusters"))
        d["gracefulEvictionTasks"] = [{"fromCluster": self.ev(t.get("FromCluster", ""))}
                                      for t in (s.get("GracefulEvictionTasks").values()
                                                if s.get("GracefulEvictionTasks") is not None else [])]
        d["placement"] = self.placement(s.get("Placement"))
        if status is not None:
            d["schedulerObservedAffinityName"] = self.ev(status.get("SchedulerObservedAffinityName", ""))
        return d

    # -- components ----------------------------------------------------------------------
    def components(self, v):
        """[]workv1alpha2.Component -> [{name, replicas, replicaRequirements?: {resourceRequest}}]."""
        out = []
        for c in (v.values() if v is not None else []):
            if isinstance(c, Call) and c.fn in self.syms and callable(self.syms[c.fn]):
                out.append(self.syms[c.fn](*c.args))
                continue
            d = {"name": self.ev(c.get("Name", "")), "replicas": self.ev(c.get("Replicas", 0))}
            rr = c.get("ReplicaRequirements")
            if rr is not None:
                d["replicaRequirements"] = {"resourceRequest": self.qmap(rr.get("ResourceRequest"))}
            out.append(d)
        return out

    # -- cluster -------------------------------------------------------------------------
    def cluster(self, c):
        if isinstance(c, dict):
            return c
        if isinstance(c, (Call, Ref)):
            c = self.ev(c)
            if isinstance(c, dict):
                return c
        d = {"name": ""}
        om = c.get("ObjectMeta")
        if om is not None:
            d["name"] = self.ev(om.get("Name", ""))
            d["labels"] = self.strmap(om.get("Labels"))
            if om.get("DeletionTimestamp") is not None:
                d["deleting"] = True
        sp = c.get("Spec")
        if sp is not None:
            d["provider"] = self.ev(sp.get("Provider", ""))
            d["region"] = self.ev(sp.get("Region", ""))
            d["zone"] = self.ev(sp.get("Zone", ""))
            d["zones"] = self.strs(sp.get("Zones"))
            d["taints"] = [{"key": self.ev(t.get("Key", "")), "value": self.ev(t.get("Value", "")),
                            "effect": self.ev(t.get("Effect", ""))}
                           for t in (sp.get("Taints").values() if sp.get("Taints") is not None else [])]
            d["resourceModels"] = [
                {"grade": self.ev(m.get("Grade", 0)),
                 "ranges": [{"name": self.key(r.get("Name", "")), "min": str(self.ev(r.get("Min", "0"))),
                             "max": str(self.ev(r.get("Max", "0")))}
                            for r in (m.get("Ranges").values() if m.get("Ranges") is not None else [])]}
                for m in (sp.get("ResourceModels").values() if sp.get("ResourceModels") is not None else [])]
        st = c.get("Status")
        if st is not None:
            ae = []
            for e in (st.get("APIEnablements").values() if st.get("APIEnablements") is not None else []):
                ae.append({"groupVersion": self.ev(e.get("GroupVersion", "")),
                           "resources": [{"kind": self.ev(x.get("Kind", ""))}
                                         for x in (e.get("Resources").values() if e.get("Resources") else [])]})
            d["apiEnablements"] = ae
            rs = st.get("ResourceSummary")
            if rs is not None:
                d["resourceSummary"] = {"allocatable": self.qmap(rs.get("Allocatable")),
                                        "allocated": self.qmap(rs.get("Allocated")),
                                        "allocating": self.qmap(rs.get("Allocating")),
                                        "allocatableModelings": [
                                            {"grade": self.ev(m.get("Grade", 0)), "count": self.ev(m.get("Count", 0))}
                                            for m in (rs.get("AllocatableModelings").values()
                                                      if rs.get("AllocatableModelings") is not None else [])]}
        return d
