"""The reference's plugin and estimator interfaces over the engine, as the Go shim in
INTEGRATION.md implements them (the Python mirror the tests drive):

  Result / Registry / Framework   framework.Result (framework/interface.go:103-211),
                                  runtime.Registry (runtime/registry.go:31-100) and the
                                  RunFilterPlugins / RunScorePlugins loops
                                  (runtime/framework.go:93-170)
  KpFilter                        framework.FilterPlugin (interface.go:85-89): answers
                                  Filter(binding, cluster) from a batch's feasibility and
                                  reason words (kp_filter_batch / kp_filter_reasons)
  KpScore                         framework.ScorePlugin (interface.go:215-223): the summed
                                  in-tree score per pair (kp_score_batch), no normalizer
  KpEstimator                     estimatorclient.ReplicaEstimator (estimator/client/
                                  interface.go:39-44): MaxAvailableReplicas through
                                  kp_max_available_replicas (clusters in request order),
                                  MaxAvailableComponentSets through
                                  kp_max_available_component_sets
  enabled_plugins_mask            `--plugins` (options.go:163) filtered over the in-tree
                                  registry (plugins/registry.go:33-50) as kp_options'
                                  enabled_plugins bitmask

A batch is keyed by binding slot: the shim computes the device arrays once per batch
and every per-pair call is a lookup. Shim mirrors the Go shim's spec -> slot index,
its estimator cache keyed by request content, and their release / invalidation. The product path is the C-ABI; nothing here
computes a filter, score or estimate itself.
"""
from __future__ import annotations

import ctypes as C
import json
from typing import Callable, Dict, List, Optional, Sequence, Tuple

from karmada_amd import api
from karmada_amd.engine import Batch, PackCache, Snapshot

SUCCESS, UNSCHEDULABLE, ERROR = 0, 1, 2  # framework.Code (interface.go:124-133)

# in-tree plugin names (plugins/registry.go:33-50) -> kp_options.enabled_plugins bits
IN_TREE = {
    "APIEnablement": api.PLUGIN_API_ENABLEMENT,
    "TaintToleration": api.PLUGIN_TAINT_TOLERATION,
    "ClusterAffinity": api.PLUGIN_CLUSTER_AFFINITY,
    "SpreadConstraint": api.PLUGIN_SPREAD_CONSTRAINT,
    "ClusterLocality": api.PLUGIN_CLUSTER_LOCALITY,
    "ClusterEviction": api.PLUGIN_CLUSTER_EVICTION,
}


class Result:
    """framework.Result: a code and reasons; None stands for Success (interface.go:175-177)."""

    def __init__(self, code: int = SUCCESS, *reasons: str):
        self.code = code
        self.reasons = list(reasons)

    def is_success(self) -> bool:
        return self.code == SUCCESS

    def __repr__(self):
        return f"Result({self.code}, {self.reasons})"


def is_success(r: Optional[Result]) -> bool:
    return r is None or r.is_success()


class Registry(dict):
    """runtime.Registry: plugin name -> factory (registry.go:31-100)."""

    def register(self, name: str, factory: Callable):
        if name in self:
            raise ValueError(f"a plugin named {name} already exists")
        self[name] = factory

    def unregister(self, name: str):
        if name not in self:
            raise ValueError(f"no plugin named {name} exists")
        del self[name]

    def merge(self, other: "Registry"):
        for k, f in other.items():
            self.register(k, f)

    def factory_names(self) -> List[str]:
        return sorted(self)

    def filter(self, names: Sequence[str]) -> "Registry":
        """--plugins: '*' enables every plugin, 'foo' enables foo, '-foo' disables it
        (registry.go:74-100; a '-foo' before any plugin is enabled has no effect)."""
        out = Registry()
        if "*" in names:
            out.update(self)
        for n in names:
            if n in self:
                out[n] = self[n]
                continue
            if n.startswith("-") and len(out) > 0:
                out.pop(n.lstrip("-"), None)
        return out


def enabled_plugins_mask(names: Sequence[str]) -> int:
    """kp_options.enabled_plugins for a `--plugins` flag value over the in-tree registry."""
    reg = Registry({k: None for k in IN_TREE})
    m = 0
    for k in reg.filter(names):
        m |= IN_TREE[k]
    return m


class Framework:
    """frameworkImpl (runtime/framework.go:64-184): the filter plugins run in order with
    a short circuit on the first non-success Result; the score plugins' scores are
    collected per plugin, with NormalizeScore when a plugin has ScoreExtensions."""

    def __init__(self, registry: Registry):
        self.filter_plugins, self.score_plugins = [], []
        for name in registry.factory_names():
            p = registry[name]()
            if hasattr(p, "filter"):
                self.filter_plugins.append(p)
            if hasattr(p, "score"):
                self.score_plugins.append(p)

    def run_filter_plugins(self, ctx) -> Optional[Result]:
        for p in self.filter_plugins:
            r = p.filter(ctx)
            if not is_success(r):
                return r
        return Result(SUCCESS)

    def run_score_plugins(self, spec, clusters) -> Tuple[Optional[Dict[str, List[Tuple[object, int]]]], Optional[Result]]:
        """(PluginToClusterScores, nil) or (nil, an Error Result); weights are all 1
        (scorePluginsWeightMap is never populated, framework.go:41,156)."""
        out = {}
        for p in self.score_plugins:
            scores = []
            for c in clusters:
                s, r = p.score(spec, c)
                if not is_success(r):
                    return None, Result(ERROR, f"plugin {p.name()!r} failed with: {r.reasons}")
                scores.append((c, s))
            ext = p.score_extensions() if hasattr(p, "score_extensions") else None
            if ext is not None:
                r = ext.normalize_score(scores)
                if not is_success(r):
                    return None, Result(ERROR, f"plugin {p.name()!r} normalizeScore failed with: {r.reasons}")
            out[p.name()] = scores
        return out, None


class UnknownCluster(KeyError):
    """A cluster name the engine's snapshot does not hold (added since the last
    update): an error, never a silent answer for some other cluster."""


class BatchView:
    """One batch's device answers, fetched on first use and looked up per (binding
    slot, cluster). The filter reasons and the scores are separate device passes
    (kp_filter_reasons, kp_score_batch), each run only when a Filter or Score asks:
    a view that only answers the estimator (kp_max_available_replicas runs its own
    pass over the one binding) never runs them. `clusters` are the snapshot's
    cluster dicts in caller order (for taint reasons)."""

    def __init__(self, snap: Snapshot, batch: Batch, clusters: Optional[Sequence[dict]] = None):
        self.snap, self.batch, self.clusters = snap, batch, clusters
        self.C = len(snap.names)
        self.index = {n: i for i, n in enumerate(snap.names)}
        self._reasons = self._scores = None
        self.passes = []  # device passes run on this view, in order (for the tests)

    @property
    def reasons(self):
        if self._reasons is None:
            eng = self.snap.engine
            r = (C.c_uint32 * max(1, self.batch.n * self.C))()
            eng._check(eng.L.kp_filter_reasons(eng.h, self.batch.h, r), "kp_filter_reasons")
            self._reasons = r
            self.passes.append("kp_filter_reasons")
        return self._reasons

    @property
    def scores(self):
        if self._scores is None:
            eng = self.snap.engine
            r = (C.c_int64 * max(1, self.batch.n * self.C))()
            eng._check(eng.L.kp_score_batch(eng.h, self.batch.h, r), "kp_score_batch")
            self._scores = r
            self.passes.append("kp_score_batch")
        return self._scores

    def cluster_index(self, cluster: str) -> int:
        i = self.index.get(cluster)
        if i is None:
            raise UnknownCluster(f"cluster {cluster!r} is not in the engine's snapshot")
        return i

    def reason(self, slot: int, cluster: str) -> int:
        return int(self.reasons[slot * self.C + self.cluster_index(cluster)])

    def score(self, slot: int, cluster: str) -> int:
        return int(self.scores[slot * self.C + self.cluster_index(cluster)])


class KpFilter:
    """FilterPlugin answering every in-tree filter at once from the batch (register it
    with the in-tree filters disabled: --plugins=*,-APIEnablement,...). ctx = (slot,
    cluster name). A deleting cluster is skipped by findClustersThatFit before any
    plugin runs (generic_scheduler.go:138-142); here it reads as Success."""

    def __init__(self, view: BatchView):
        self.view = view

    def name(self) -> str:
        return "KpFilter"

    def filter(self, ctx) -> Optional[Result]:
        slot, cluster = ctx
        try:
            w = self.view.reason(slot, cluster)
        except UnknownCluster as err:  # framework.AsResult(err): an Error Result
            return Result(ERROR, str(err.args[0]))
        code = w & 0xFF
        if code in (api.REASON_FIT, api.REASON_DELETING):
            return None
        cl = self.view.clusters[self.view.index[cluster]] if self.view.clusters is not None else {"taints": []}
        return Result(UNSCHEDULABLE, api.reason_text(w, cl))


class KpScore:
    """ScorePlugin: the summed in-tree score (ClusterLocality + ClusterAffinity's 0)."""

    def __init__(self, view: BatchView):
        self.view = view

    def name(self) -> str:
        return "KpScore"

    def score(self, spec, cluster) -> Tuple[int, Optional[Result]]:
        try:
            return self.view.score(spec, cluster), None
        except UnknownCluster as err:
            return 0, Result(ERROR, str(err.args[0]))

    def score_extensions(self):
        return None


class KpEstimator:
    """ReplicaEstimator for the GeneralEstimator's place in GetReplicaEstimators()."""

    def __init__(self, snap: Snapshot, batch: Optional[Batch]):
        self.snap, self.batch = snap, batch

    def _indices(self, clusters: Sequence[str]) -> List[int]:
        idx = {n: i for i, n in enumerate(self.snap.names)}
        bad = [n for n in clusters if n not in idx]
        if bad:
            raise UnknownCluster(f"cluster {bad[0]!r} is not in the engine's snapshot")
        return [idx[n] for n in clusters]

    def max_available_replicas(self, slot: int, clusters: Sequence[str]) -> List[Tuple[str, int]]:
        """[]TargetCluster in the request's cluster order (general.go:57-64)."""
        eng = self.snap.engine
        ci = (C.c_uint32 * max(1, len(clusters)))(*self._indices(clusters))
        if not clusters:
            return []
        out = (C.c_int32 * max(1, len(clusters)))()
        eng._check(eng.L.kp_max_available_replicas(eng.h, self.batch.h, slot, ci, len(clusters), out),
                   "kp_max_available_replicas")
        return [(n, int(out[i])) for i, n in enumerate(clusters)]

    def max_available_component_sets(self, components: Sequence[dict], clusters: Sequence[str]) -> List[Tuple[str, int]]:
        """[]ComponentSetEstimationResponse in request order (general.go:154-162)."""
        eng = self.snap.engine
        w = api.World()
        ci = (C.c_uint32 * max(1, len(clusters)))(*self._indices(clusters))
        if not clusters:  # (the Go shim's guard before &idx[0])
            return []
        ca, nc = w.components(components)
        out = (C.c_int32 * max(1, len(clusters)))()
        eng._check(eng.L.kp_max_available_component_sets(eng.h, self.snap.h, ca, nc, ci, len(clusters), out),
                   "kp_max_available_component_sets")
        return [(n, int(out[i])) for i, n in enumerate(clusters)]


def out_of_tree_plugins(registry_names: Sequence[str], shim_name: str = "KpPlacement") -> int:
    """kp_options.n_out_of_tree_plugins: the registered plugins that are neither in-tree
    nor the shim itself (RunFilterPlugins / RunScorePlugins would run them too)."""
    return sum(1 for n in registry_names if n not in IN_TREE and n != shim_name)


def requirements_key(requirements: Optional[dict]) -> str:
    """The estimator cache key of a ReplicaRequirements: its content, canonically
    ordered (two requests with equal content share one device answer)."""
    return json.dumps(requirements, sort_keys=True, separators=(",", ":"))


class Shim:
    """The Go shim's state (plugins.go): the engine, the current
    snapshot, the spec -> (view, slot) index of the batches packed this cycle, and the
    estimator's requirements -> (view, slot) cache.

    * schedule_batch(specs) packs and schedules a batch (ScheduleBatch) and registers
      every spec of it, so Filter/Score for those specs are lookups;
    * slot_of(spec) finds a spec by identity (the Go map is keyed by *ResourceBindingSpec);
      an unseen spec is packed as a one-binding batch once;
    * max_available_replicas(requirements, clusters) answers from a one-binding batch
      per distinct requirements content, reused by every later equal request;
    * release(specs) ends those specs' cycle: a view whose specs are all released is
      destroyed (kp_batch_destroy);
    * update(clusters) applies cluster events and destroys every view (their device
      arrays describe the old snapshot).
    The batch path refuses a registry with out-of-tree filter/score plugins
    (kp_options.n_out_of_tree_plugins, KP_ENOTSUP); the per-pair answers stay available.
    """

    def __init__(self, engine, clusters: Sequence[dict], opts: Optional[api.kp_options] = None,
                 registry_names: Sequence[str] = ()):
        # a copy: the caller's kp_options stays as it was (reusing it for another
        # snapshot must not carry this shim's out-of-tree count)
        opts = api.kp_options.from_buffer_copy(opts) if opts is not None else api.options()
        opts.n_out_of_tree_plugins = out_of_tree_plugins(registry_names)
        self.clusters = list(clusters)
        self.snap = Snapshot(engine, self.clusters, opts)
        self.by: Dict[int, Tuple[BatchView, int]] = {}   # id(spec) -> (view, slot)
        self.keep: Dict[int, dict] = {}                  # id(spec) -> spec (ids stay unique while held)
        self.est: Dict[str, Tuple[BatchView, int]] = {}  # requirements content -> (view, slot)
        self.live: Dict[int, int] = {}                   # id(view) -> specs still registered
        self.batches_created = 0
        # packed records kept across cycles, keyed by (uid, metadata.generation): the Go
        # shim's kp_pack_cache (INTEGRATION.md ScheduleBatchKeyed)
        self.pack_cache = PackCache(engine)

    def _view(self, specs: Sequence[dict], generations: Optional[Sequence[int]] = None) -> BatchView:
        if generations is None:
            b = Batch(self.snap, list(specs))
        else:
            b = Batch(self.snap, list(specs), cache=self.pack_cache, generations=generations)
        self.batches_created += 1
        return BatchView(self.snap, b, self.clusters)

    def _register(self, view: BatchView, specs: Sequence[dict]):
        for i, sp in enumerate(specs):
            self.by[id(sp)] = (view, i)
            self.keep[id(sp)] = sp
        self.live[id(view)] = self.live.get(id(view), 0) + len(specs)

    def schedule_batch(self, specs: Sequence[dict], generations: Optional[Sequence[int]] = None) -> List[dict]:
        """ScheduleBatch; with `generations` (metadata.generation per spec, the spec's "uid"
        as the other half of the key) ScheduleBatchKeyed: records of unchanged bindings
        are reused from earlier cycles instead of re-packed (kp_batch_create_keyed)."""
        view = self._view(specs, generations)
        self._register(view, specs)
        return view.batch.schedule()

    def slot_of(self, spec: dict) -> Tuple[BatchView, int]:
        hit = self.by.get(id(spec))
        if hit is not None and self.keep.get(id(spec)) is spec:
            return hit
        view = self._view([spec])
        self._register(view, [spec])
        return view, 0

    def filter(self, spec: dict, cluster: str) -> Optional[Result]:
        view, slot = self.slot_of(spec)
        return KpFilter(view).filter((slot, cluster))

    def score(self, spec: dict, cluster: str) -> Tuple[int, Optional[Result]]:
        view, slot = self.slot_of(spec)
        return KpScore(view).score(slot, cluster)

    def max_available_replicas(self, requirements: Optional[dict], clusters: Sequence[str]) -> List[Tuple[str, int]]:
        key = requirements_key(requirements)
        hit = self.est.get(key)
        if hit is None:
            spec = {"replicas": 1}
            if requirements is not None:
                spec["replicaRequirements"] = requirements
            view = self._view([spec])
            hit = self.est[key] = (view, 0)
        view, slot = hit
        return KpEstimator(self.snap, view.batch).max_available_replicas(slot, clusters)

    def release(self, specs: Sequence[dict]):
        for sp in specs:
            hit = self.by.pop(id(sp), None)
            self.keep.pop(id(sp), None)
            if hit is None:
                continue
            view = hit[0]
            self.live[id(view)] -= 1
            if self.live[id(view)] == 0:
                del self.live[id(view)]
                view.batch.close()

    def update(self, clusters: Sequence[dict]) -> bool:
        grew = self.snap.update(clusters)
        by_name = {c["name"]: c for c in clusters}
        self.clusters = [by_name.get(c["name"], c) for c in self.clusters]
        for view, _ in list(self.by.values()) + list(self.est.values()):
            view.batch.close()
        self.by.clear()
        self.keep.clear()
        self.est.clear()
        self.live.clear()
        return grew

    def close(self):
        for view, _ in list(self.by.values()) + list(self.est.values()):
            view.batch.close()
        self.by.clear()
        self.est.clear()
        self.pack_cache.close()
        self.snap.close()
