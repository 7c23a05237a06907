"""ctypes mirror of include/kp/kp_api.h and builders from Karmada-style dicts.

The dict layout follows the JSON field names of the reference API types
(pkg/apis/cluster/v1alpha1/types.go, pkg/apis/work/v1alpha2/binding_types.go,
pkg/apis/policy/v1alpha1/propagation_types.go) so that table-driven tests read
like the reference's own tests. A `World` keeps every ctypes buffer alive for
as long as the C structs that point into it are in use.
"""
from __future__ import annotations

import ctypes as C
from typing import Any, Dict, List, Optional, Sequence

u8, u32, i32, i64, u64 = C.c_uint8, C.c_uint32, C.c_int32, C.c_int64, C.c_uint64


class kp_str(C.Structure):
    _fields_ = [("ptr", C.c_char_p), ("len", u32)]


class kp_label(C.Structure):
    _fields_ = [("key", kp_str), ("value", kp_str)]


class kp_requirement(C.Structure):
    _fields_ = [("key", kp_str), ("op", kp_str), ("values", C.POINTER(kp_str)), ("n_values", u32)]


class kp_cluster_affinity(C.Structure):
    _fields_ = [
        ("has_label_selector", u8),
        ("match_labels", C.POINTER(kp_label)), ("n_match_labels", u32),
        ("match_expressions", C.POINTER(kp_requirement)), ("n_match_expressions", u32),
        ("has_field_selector", u8),
        ("field_expressions", C.POINTER(kp_requirement)), ("n_field_expressions", u32),
        ("cluster_names", C.POINTER(kp_str)), ("n_cluster_names", u32),
        ("exclude_clusters", C.POINTER(kp_str)), ("n_exclude_clusters", u32),
    ]


class kp_affinity_term(C.Structure):
    _fields_ = [("affinity_name", kp_str), ("affinity", kp_cluster_affinity),
                ("overflow", C.POINTER(kp_cluster_affinity)), ("n_overflow", u32)]


class kp_toleration(C.Structure):
    _fields_ = [("key", kp_str), ("op", kp_str), ("value", kp_str), ("effect", kp_str)]


class kp_taint(C.Structure):
    _fields_ = [("key", kp_str), ("value", kp_str), ("effect", kp_str)]


class kp_spread_constraint(C.Structure):
    _fields_ = [("spread_by_field", kp_str), ("spread_by_label", kp_str),
                ("max_groups", i64), ("min_groups", i64)]


class kp_static_weight(C.Structure):
    _fields_ = [("target", kp_cluster_affinity), ("weight", i64)]


class kp_resource(C.Structure):
    _fields_ = [("name", kp_str), ("quantity", kp_str)]


class kp_target_cluster(C.Structure):
    _fields_ = [("name", kp_str), ("replicas", i32)]


class kp_component(C.Structure):
    _fields_ = [("name", kp_str), ("replicas", i32), ("has_replica_requirements", u8),
                ("resource_request", C.POINTER(kp_resource)), ("n_resource_request", u32)]


class kp_binding(C.Structure):
    _fields_ = [
        ("uid", kp_str), ("api_version", kp_str), ("kind", kp_str), ("namespace_", kp_str), ("name", kp_str),
        ("replicas", i32),
        ("has_replica_requirements", u8), ("has_node_claim", u8),
        ("resource_request", C.POINTER(kp_resource)), ("n_resource_request", u32),
        ("n_components", u32), ("components", C.POINTER(kp_component)),
        ("clusters", C.POINTER(kp_target_cluster)), ("n_clusters", u32),
        ("eviction_from", C.POINTER(kp_str)), ("n_eviction_from", u32),
        ("has_reschedule_triggered_at", u8), ("has_last_scheduled_time", u8),
        ("reschedule_triggered_at_ns", i64), ("last_scheduled_time_ns", i64),
        ("observed_affinity_name", kp_str),
        ("has_cluster_affinity", u8), ("cluster_affinity", kp_cluster_affinity),
        ("cluster_affinities", C.POINTER(kp_affinity_term)), ("n_cluster_affinities", u32),
        ("tolerations", C.POINTER(kp_toleration)), ("n_tolerations", u32),
        ("spread_constraints", C.POINTER(kp_spread_constraint)), ("n_spread_constraints", u32),
        ("has_replica_scheduling", u8), ("replica_scheduling_type", kp_str),
        ("replica_division_preference", kp_str),
        ("has_weight_preference", u8),
        ("static_weights", C.POINTER(kp_static_weight)), ("n_static_weights", u32),
        ("dynamic_weight", kp_str),
    ]


class kp_api_enablement(C.Structure):
    _fields_ = [("group_version", kp_str), ("kind", kp_str)]


class kp_model_range(C.Structure):
    _fields_ = [("name", kp_str), ("min", kp_str), ("max", kp_str)]


class kp_resource_model(C.Structure):
    _fields_ = [("grade", u32), ("ranges", C.POINTER(kp_model_range)), ("n_ranges", u32)]


class kp_node(C.Structure):
    _fields_ = [("name", kp_str), ("labels", C.POINTER(kp_label)), ("n_labels", u32),
                ("taints", C.POINTER(kp_taint)), ("n_taints", u32), ("unschedulable", i32),
                ("allocatable", C.POINTER(kp_resource)), ("n_allocatable", u32),
                ("requested", C.POINTER(kp_resource)), ("n_requested", u32), ("n_pods", u32)]


class kp_node_selector_term(C.Structure):
    _fields_ = [("match_expressions", C.POINTER(kp_requirement)), ("n_match_expressions", u32),
                ("match_fields", C.POINTER(kp_requirement)), ("n_match_fields", u32)]


class kp_node_claim(C.Structure):
    _fields_ = [("node_selector", C.POINTER(kp_label)), ("n_node_selector", u32),
                ("tolerations", C.POINTER(kp_toleration)), ("n_tolerations", u32),
                ("has_node_affinity", i32),
                ("node_affinity_terms", C.POINTER(kp_node_selector_term)), ("n_node_affinity_terms", u32)]


class kp_node_component(C.Structure):
    _fields_ = [("replicas", i32), ("has_replica_requirements", u8),
                ("resource_request", C.POINTER(kp_resource)), ("n_resource_request", u32),
                ("node_claim", C.POINTER(kp_node_claim))]


class kp_assumed_workload(C.Structure):
    _fields_ = [("components", C.POINTER(kp_node_component)), ("n_components", u32)]


class kp_allocatable_modeling(C.Structure):
    _fields_ = [("grade", u32), ("count", i64)]


class kp_cluster(C.Structure):
    _fields_ = [
        ("name", kp_str), ("deleting", u8),
        ("labels", C.POINTER(kp_label)), ("n_labels", u32),
        ("provider", kp_str), ("region", kp_str), ("zone", kp_str),
        ("zones", C.POINTER(kp_str)), ("n_zones", u32),
        ("taints", C.POINTER(kp_taint)), ("n_taints", u32),
        ("api_enablements", C.POINTER(kp_api_enablement)), ("n_api_enablements", u32),
        ("resource_models", C.POINTER(kp_resource_model)), ("n_resource_models", u32),
        ("has_resource_summary", u8),
        ("allocatable", C.POINTER(kp_resource)), ("n_allocatable", u32),
        ("allocated", C.POINTER(kp_resource)), ("n_allocated", u32),
        ("allocating", C.POINTER(kp_resource)), ("n_allocating", u32),
        ("allocatable_modelings", C.POINTER(kp_allocatable_modeling)), ("n_allocatable_modelings", u32),
    ]


class kp_options(C.Structure):
    _fields_ = [("enable_empty_workload_propagation", u8),
                ("customized_cluster_resource_modeling", u8),
                ("multiple_pod_templates_scheduling", u8),
                ("enabled_plugins", u32),
                ("n_out_of_tree_plugins", u32)]


class kp_results(C.Structure):
    _fields_ = [("n_bindings", u64), ("status", C.POINTER(i32)), ("err_code", C.POINTER(i32)),
                ("err_arg", C.POINTER(i64)), ("offsets", C.POINTER(u64)),
                ("cluster_idx", C.POINTER(u32)), ("replicas", C.POINTER(i32)), ("n_targets", u64)]


class kp_binding_key(C.Structure):
    _fields_ = [("uid", kp_str), ("generation", i64)]


class kp_pack_cache_stats(C.Structure):
    _fields_ = [("hits", u64), ("misses", u64), ("entries", u64), ("last_hits", u64)]


def binding_keys(bindings, n, generations):
    """kp_binding_key per binding: its uid (kp_binding.uid, shared, not copied) and the
    given metadata.generation."""
    ks = (kp_binding_key * max(1, n))()
    for i in range(n):
        ks[i].uid = bindings[i].uid
        ks[i].generation = int(generations[i])
    return ks


class kp_affinity_results(C.Structure):
    _fields_ = [("results", kp_results), ("affinity_index", C.POINTER(i32)), ("attempts", C.POINTER(i32)),
                ("rounds", C.c_uint32)]


class kp_kernel_time(C.Structure):
    _fields_ = [("name", C.c_char * 32), ("ms", C.c_float), ("launches", u32), ("units", u64)]


class kp_stage_times(C.Structure):
    _fields_ = [("pair_ms", C.c_double), ("select_ms", C.c_double), ("host_ms", C.c_double),
                ("copy_ms", C.c_double), ("total_ms", C.c_double),
                ("pair_kernel_ms", C.c_float), ("select_kernel_ms", C.c_float), ("n_slow", u64),
                ("pair_launches", C.c_uint32), ("pair_kind", C.c_uint32),
                ("filter_kernel_ms", C.c_float), ("bits", C.c_uint32),
                ("sel_all_kernel_ms", C.c_float), ("n_sel_all", C.c_uint32),
                ("n_classes", C.c_uint32), ("n_top", C.c_uint32), ("n_top_fallback", C.c_uint32),
                ("top_kernel_ms", C.c_float), ("n_cluster", C.c_uint32), ("n_cluster_order", C.c_uint32),
                ("cluster_kernel_ms", C.c_float), ("n_region", C.c_uint32), ("n_region_order", C.c_uint32)]


PLUGIN_API_ENABLEMENT = 1 << 0
PLUGIN_TAINT_TOLERATION = 1 << 1
PLUGIN_CLUSTER_AFFINITY = 1 << 2
PLUGIN_SPREAD_CONSTRAINT = 1 << 3
PLUGIN_CLUSTER_LOCALITY = 1 << 4
PLUGIN_CLUSTER_EVICTION = 1 << 5
PLUGIN_ALL = 0x3F

STATUS_OK, STATUS_FIT_ERROR, STATUS_UNSCHEDULABLE, STATUS_ERROR = 0, 1, 2, 3

# kp_filter_reasons codes (kp_api.h KP_REASON_*) and the Result reasons the plugins return
REASON_FIT, REASON_API, REASON_TAINT, REASON_AFFINITY = 0, 1, 2, 3
REASON_SPREAD_PROVIDER, REASON_SPREAD_REGION, REASON_SPREAD_ZONES, REASON_EVICTION = 4, 5, 6, 7
REASON_DELETING = 255
REASON_TEXT = {
    REASON_API: "cluster(s) did not have the API resource",                              # api_enablement.go:77
    REASON_TAINT: "cluster(s) had untolerated taint {%s}",                               # taint_toleration.go:83
    REASON_AFFINITY: "cluster(s) did not match the placement cluster affinity constraint",  # cluster_affinity.go:89
    REASON_SPREAD_PROVIDER: "cluster(s) did not have provider property",                 # spread_constraint.go:57
    REASON_SPREAD_REGION: "cluster(s) did not have region property",                     # spread_constraint.go:59
    REASON_SPREAD_ZONES: "cluster(s) did not have zones property",                       # spread_constraint.go:61
    REASON_EVICTION: "cluster(s) is in the process of eviction",                         # cluster_eviction.go:53
}


def taint_string(t: dict) -> str:
    """corev1.Taint.ToString()."""
    if not t.get("value"):
        return "%s:%s" % (t.get("key", ""), t.get("effect", ""))
    return "%s=%s:%s" % (t.get("key", ""), t.get("value", ""), t.get("effect", ""))


def reason_text(code: int, cluster: dict) -> str:
    """The Result reason of one kp_filter_reasons word for `cluster` (its dict form)."""
    kind, arg = code & 0xFF, code >> 8
    if kind == REASON_TAINT:
        taints = [t for t in cluster.get("taints", []) if t.get("effect") in ("NoSchedule", "NoExecute")]
        return REASON_TEXT[kind] % taint_string(taints[arg])
    return REASON_TEXT[kind]


def fit_error_message(num_all_clusters: int, reasons: dict) -> str:
    """FitError.Error() (framework/types.go:67-91): reasons = {cluster name: reason text or
    list of texts} for the clusters of Diagnosis.ClusterToResultMap."""
    if num_all_clusters == 0 or not reasons:
        return "0/%d clusters are available: %s." % (num_all_clusters, "no cluster exists")
    hist = {}
    for rs in reasons.values():
        for r in ([rs] if isinstance(rs, str) else rs):
            hist[r] = hist.get(r, 0) + 1
    return "0/%d clusters are available: %s." % (num_all_clusters,
                                                   ", ".join(sorted("%d %s" % (v, k) for k, v in hist.items())))
ERR_NAMES = {
    0: "none", 1: "fit", 2: "region_min_groups", 3: "region_cluster_min", 4: "cluster_min_groups",
    5: "cluster_resource", 6: "spread_unsupported", 7: "no_clusters", 8: "unsupported_strategy",
    9: "overflow_not_enough", 10: "fresh_not_enough", 11: "scale_down_not_enough",
    12: "scale_up_not_enough", 13: "undefined_strategy", 14: "result_capacity", 15: "sets_capacity",
    16: "overflow_terms",
}


def options(empty_workload_propagation=False, models_gate=True, plugins=PLUGIN_ALL,
            multi_templates=False, out_of_tree_plugins=0) -> kp_options:
    return kp_options(enable_empty_workload_propagation=int(empty_workload_propagation),
                      customized_cluster_resource_modeling=int(models_gate),
                      multiple_pod_templates_scheduling=int(multi_templates), enabled_plugins=plugins,
                      n_out_of_tree_plugins=int(out_of_tree_plugins))


class World:
    """Owns ctypes buffers; builds C structs from dicts."""

    def __init__(self) -> None:
        self._keep: List[Any] = []

    # -- primitives ------------------------------------------------------------------
    def s(self, v: Optional[str]) -> kp_str:
        if not v:
            return kp_str(None, 0)
        b = v.encode() if isinstance(v, str) else bytes(v)
        self._keep.append(b)
        return kp_str(b, len(b))

    def arr(self, ctype, items: Sequence[Any]):
        if not items:
            return None, 0
        a = (ctype * len(items))(*items)
        self._keep.append(a)
        return a, len(items)

    def strs(self, vs: Optional[Sequence[str]]):
        return self.arr(kp_str, [self.s(v) for v in (vs or [])])

    def resources(self, rl: Optional[Dict[str, str]]):
        return self.arr(kp_resource, [kp_resource(self.s(k), self.s(str(v))) for k, v in (rl or {}).items()])

    def components(self, comps):
        """[{name, replicas, replicaRequirements?: {resourceRequest}}] -> (kp_component array, n)."""
        out = []
        for c in comps or []:
            rr = c.get("replicaRequirements")
            ra, nr = self.resources((rr or {}).get("resourceRequest"))
            out.append(kp_component(self.s(c.get("name", "")), int(c.get("replicas", 0)), 1 if rr is not None else 0,
                                    ra, nr))
        return self.arr(kp_component, out)

    def requirements(self, exprs):
        out = []
        for e in exprs or []:
            vals, nv = self.strs(e.get("values"))
            out.append(kp_requirement(self.s(e["key"]), self.s(e["operator"]), vals, nv))
        return self.arr(kp_requirement, out)

    def affinity(self, a: Optional[dict]) -> kp_cluster_affinity:
        r = kp_cluster_affinity()
        if not a:
            return r
        ls = a.get("labelSelector")
        if ls is not None:
            r.has_label_selector = 1
            ml = [kp_label(self.s(k), self.s(v)) for k, v in (ls.get("matchLabels") or {}).items()]
            r.match_labels, r.n_match_labels = self.arr(kp_label, ml)
            r.match_expressions, r.n_match_expressions = self.requirements(ls.get("matchExpressions"))
        fs = a.get("fieldSelector")
        if fs is not None:
            r.has_field_selector = 1
            r.field_expressions, r.n_field_expressions = self.requirements(fs.get("matchExpressions"))
        r.cluster_names, r.n_cluster_names = self.strs(a.get("clusterNames"))
        r.exclude_clusters, r.n_exclude_clusters = self.strs(a.get("exclude"))
        return r

    def models(self, ms):
        """[{grade, ranges: [{name, min, max}]}] -> (kp_resource_model array, n)."""
        out = []
        for m in ms or []:
            rr = [kp_model_range(self.s(r["name"]), self.s(str(r.get("min", "0"))), self.s(str(r.get("max", ""))))
                  for r in m.get("ranges") or []]
            ra, nr = self.arr(kp_model_range, rr)
            out.append(kp_resource_model(m.get("grade", 0), ra, nr))
        return self.arr(kp_resource_model, out)

    # -- member-cluster node ------------------------------------------------------------
    def node(self, d: dict) -> kp_node:
        """{name, labels, taints, unschedulable, allocatable, requested, pods} -> kp_node."""
        n = kp_node()
        n.name = self.s(d.get("name", ""))
        n.labels, n.n_labels = self.arr(kp_label, [kp_label(self.s(k), self.s(v)) for k, v in (d.get("labels") or {}).items()])
        n.taints, n.n_taints = self.arr(kp_taint, [
            kp_taint(self.s(t.get("key")), self.s(t.get("value")), self.s(t.get("effect"))) for t in d.get("taints") or []])
        n.unschedulable = int(bool(d.get("unschedulable")))
        n.allocatable, n.n_allocatable = self.resources(d.get("allocatable"))
        n.requested, n.n_requested = self.resources(d.get("requested"))
        n.n_pods = int(d.get("pods", 0))
        return n

    def nodes(self, ds):
        a = (kp_node * max(1, len(ds)))(*[self.node(d) for d in ds])
        self._keep.append(a)
        return a, len(ds)

    def node_claim(self, d: Optional[dict]):
        """{nodeSelector: {k: v}, tolerations: [...], nodeAffinity: {nodeSelectorTerms: [{matchExpressions,
        matchFields}]}} -> kp_node_claim or None (nodeAffinity: the NodeSelector that NodeAffinityBytes holds)."""
        if d is None:
            return None
        c = kp_node_claim()
        c.node_selector, c.n_node_selector = self.arr(kp_label, [
            kp_label(self.s(k), self.s(v)) for k, v in (d.get("nodeSelector") or {}).items()])
        c.tolerations, c.n_tolerations = self.arr(kp_toleration, [
            kp_toleration(self.s(t.get("key")), self.s(t.get("operator")), self.s(t.get("value")), self.s(t.get("effect")))
            for t in d.get("tolerations") or []])
        na = d.get("nodeAffinity")
        c.has_node_affinity = int(na is not None)
        terms = []
        for t in (na or {}).get("nodeSelectorTerms") or []:
            me, nme = self.requirements(t.get("matchExpressions"))
            mf, nmf = self.requirements(t.get("matchFields"))
            terms.append(kp_node_selector_term(me, nme, mf, nmf))
        c.node_affinity_terms, c.n_node_affinity_terms = self.arr(kp_node_selector_term, terms)
        self._keep.append(c)
        return c

    def node_components(self, comps):
        """pb.Component dicts {replicas, replicaRequirements: {resourceRequest, nodeClaim}} -> kp_node_component[]."""
        out = []
        for c in comps or []:
            rr = c.get("replicaRequirements")
            ra, nr = self.resources((rr or {}).get("resourceRequest"))
            nc = self.node_claim((rr or {}).get("nodeClaim"))
            out.append(kp_node_component(int(c.get("replicas", 0)), 1 if rr is not None else 0, ra, nr,
                                         C.pointer(nc) if nc is not None else None))
        return self.arr(kp_node_component, out)

    def assumed_workloads(self, ws):
        """pb.AssumedWorkload dicts {components: [...]} -> kp_assumed_workload[]."""
        out = []
        for w in ws or []:
            ca, nc = self.node_components(w.get("components"))
            out.append(kp_assumed_workload(ca, nc))
        return self.arr(kp_assumed_workload, out)

    # -- cluster ---------------------------------------------------------------------
    def cluster(self, d: dict) -> kp_cluster:
        c = kp_cluster()
        c.name = self.s(d["name"])
        c.deleting = int(bool(d.get("deleting")))
        c.labels, c.n_labels = self.arr(kp_label, [kp_label(self.s(k), self.s(v)) for k, v in (d.get("labels") or {}).items()])
        c.provider, c.region, c.zone = self.s(d.get("provider")), self.s(d.get("region")), self.s(d.get("zone"))
        c.zones, c.n_zones = self.strs(d.get("zones"))
        c.taints, c.n_taints = self.arr(kp_taint, [
            kp_taint(self.s(t.get("key")), self.s(t.get("value")), self.s(t.get("effect"))) for t in d.get("taints") or []])
        apis = []
        for e in d.get("apiEnablements") or []:
            for r in e.get("resources") or []:
                apis.append(kp_api_enablement(self.s(e.get("groupVersion")), self.s(r.get("kind"))))
        c.api_enablements, c.n_api_enablements = self.arr(kp_api_enablement, apis)
        models = []
        for m in d.get("resourceModels") or []:
            rr = [kp_model_range(self.s(r["name"]), self.s(str(r.get("min", "0"))), self.s(str(r.get("max", ""))))
                  for r in m.get("ranges") or []]
            ra, nr = self.arr(kp_model_range, rr)
            models.append(kp_resource_model(m.get("grade", 0), ra, nr))
        c.resource_models, c.n_resource_models = self.arr(kp_resource_model, models)
        rs = d.get("resourceSummary")
        if rs is not None:
            c.has_resource_summary = 1
            c.allocatable, c.n_allocatable = self.resources(rs.get("allocatable"))
            c.allocated, c.n_allocated = self.resources(rs.get("allocated"))
            c.allocating, c.n_allocating = self.resources(rs.get("allocating"))
            c.allocatable_modelings, c.n_allocatable_modelings = self.arr(kp_allocatable_modeling, [
                kp_allocatable_modeling(m.get("grade", 0), m.get("count", 0)) for m in rs.get("allocatableModelings") or []])
        return c

    def clusters(self, ds: Sequence[dict]):
        a = (kp_cluster * max(1, len(ds)))(*[self.cluster(d) for d in ds])
        self._keep.append(a)
        return a, len(ds)

    # -- binding ---------------------------------------------------------------------
    def binding(self, d: dict) -> kp_binding:
        b = kp_binding()
        b.uid = self.s(d.get("uid"))
        b.api_version = self.s(d.get("apiVersion", "apps/v1"))
        b.kind = self.s(d.get("kind", "Deployment"))
        b.namespace_ = self.s(d.get("namespace", "default"))
        b.name = self.s(d.get("name", "demo"))
        b.replicas = int(d.get("replicas", 0))
        rr = d.get("replicaRequirements")
        if rr is not None:
            b.has_replica_requirements = 1
            b.resource_request, b.n_resource_request = self.resources(rr.get("resourceRequest"))
            b.has_node_claim = int(rr.get("nodeClaim") is not None)
        comps = d.get("components")
        if isinstance(comps, list):
            b.components, b.n_components = self.components(comps)
        else:
            b.n_components = int(comps or 0)
        b.clusters, b.n_clusters = self.arr(kp_target_cluster, [
            kp_target_cluster(self.s(t["name"]), int(t.get("replicas", 0))) for t in d.get("clusters") or []])
        b.eviction_from, b.n_eviction_from = self.strs([t["fromCluster"] for t in d.get("gracefulEvictionTasks") or []])
        if d.get("rescheduleTriggeredAt") is not None:
            b.has_reschedule_triggered_at = 1
            b.reschedule_triggered_at_ns = int(d["rescheduleTriggeredAt"])
        if d.get("lastScheduledTime") is not None:
            b.has_last_scheduled_time = 1
            b.last_scheduled_time_ns = int(d["lastScheduledTime"])
        b.observed_affinity_name = self.s(d.get("schedulerObservedAffinityName"))
        p = d.get("placement") or {}
        if p.get("clusterAffinity") is not None:
            b.has_cluster_affinity = 1
            b.cluster_affinity = self.affinity(p["clusterAffinity"])
        terms = []
        for t in p.get("clusterAffinities") or []:
            ov, nov = self.arr(kp_cluster_affinity, [self.affinity(o) for o in t.get("overflowAffinities") or []])
            terms.append(kp_affinity_term(self.s(t.get("affinityName")), self.affinity(t), ov, nov))
        b.cluster_affinities, b.n_cluster_affinities = self.arr(kp_affinity_term, terms)
        b.tolerations, b.n_tolerations = self.arr(kp_toleration, [
            kp_toleration(self.s(t.get("key")), self.s(t.get("operator")), self.s(t.get("value")), self.s(t.get("effect")))
            for t in p.get("clusterTolerations") or []])
        b.spread_constraints, b.n_spread_constraints = self.arr(kp_spread_constraint, [
            kp_spread_constraint(self.s(s.get("spreadByField")), self.s(s.get("spreadByLabel")),
                                 int(s.get("maxGroups", 0)), int(s.get("minGroups", 0)))
            for s in p.get("spreadConstraints") or []])
        rs = p.get("replicaScheduling")
        if rs is not None:
            b.has_replica_scheduling = 1
            b.replica_scheduling_type = self.s(rs.get("replicaSchedulingType"))
            b.replica_division_preference = self.s(rs.get("replicaDivisionPreference"))
            wp = rs.get("weightPreference")
            if wp is not None:
                b.has_weight_preference = 1
                b.static_weights, b.n_static_weights = self.arr(kp_static_weight, [
                    kp_static_weight(self.affinity(w.get("targetCluster")), int(w.get("weight", 0)))
                    for w in wp.get("staticWeightList") or []])
                b.dynamic_weight = self.s(wp.get("dynamicWeight"))
        return b

    def bindings(self, ds: Sequence[dict]):
        a = (kp_binding * max(1, len(ds)))(*[self.binding(d) for d in ds])
        self._keep.append(a)
        return a, len(ds)


def results_to_python(status, err_code, err_arg, offsets, cluster_idx, replicas, n) -> List[dict]:
    """Converts result arrays into a list of {status, err, arg, targets: sorted [(idx, rep)]}."""
    out = []
    for i in range(n):
        lo, hi = offsets[i], offsets[i + 1]
        tg = sorted((int(cluster_idx[k]), int(replicas[k])) for k in range(lo, hi))
        out.append({"status": int(status[i]), "err": int(err_code[i]), "arg": int(err_arg[i]), "targets": tg})
    return out
