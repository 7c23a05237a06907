"""Host-side mirror of the reference scheduling interface over libkp.so.

The product path: Python objects -> kp_api.h structs (api.World) -> libkp.so
(C-ABI, HIP kernels on gfx950). There is no CPU fallback: if libkp.so is
missing or no GPU is visible, construction raises.

Mirrors (reference file:line):
  GenericScheduler.schedule  <- genericScheduler.Schedule
                                 (pkg/scheduler/core/generic_scheduler.go:70-121)
  GenericScheduler.filter    <- findClustersThatFit (generic_scheduler.go:123-150)
  GenericScheduler.score     <- prioritizeClusters (generic_scheduler.go:152-181)
  GenericScheduler.max_available_replicas
                             <- estimator.ReplicaEstimator.MaxAvailableReplicas
                                 (pkg/estimator/client/interface.go:34-37) via
                                 calAvailableReplicas (core/util.go:56-118)
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

from karmada_amd import api

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG, "libkp.so")
KP_ABI_VERSION = 14

_LIBS = {}

# C-ABI entry points declared in include/kp/kp_api.h
EXPORTS = (
    "kp_abi_version", "kp_engine_create", "kp_engine_destroy", "kp_last_error", "kp_snapshot_create",
    "kp_snapshot_destroy", "kp_snapshot_export", "kp_snapshot_import", "kp_snapshot_update", "kp_batch_create",
    "kp_batch_destroy", "kp_batch_create_keyed", "kp_batch_digest", "kp_pack_cache_create", "kp_pack_cache_destroy",
    "kp_pack_cache_get_stats",
    "kp_schedule_batch", "kp_schedule_batch_submit", "kp_schedule_batch_collect", "kp_schedule_affinities", "kp_filter_batch", "kp_filter_reasons", "kp_score_batch", "kp_max_available_replicas", "kp_max_available_component_sets",
    "kp_model_grades", "kp_node_max_replicas", "kp_node_max_component_sets", "kp_last_stage_times",
    "kp_engine_set_threads", "kp_snapshot_replicate", "kp_engine_set_profile", "kp_last_kernel_times",
    "kp_multi_create", "kp_multi_destroy", "kp_multi_last_error", "kp_multi_devices", "kp_multi_engine",
    "kp_multi_snapshot_create", "kp_multi_snapshot_update", "kp_multi_snapshot_destroy", "kp_multi_snapshot_replica",
    "kp_multi_shard_cuts", "kp_multi_batch_create", "kp_multi_batch_destroy", "kp_multi_batch_shards",
    "kp_multi_schedule",
)

KP_OK, KP_EINVAL, KP_ENOMEM, KP_EDEVICE, KP_ENOTSUP, KP_ESTATE = 0, -1, -2, -3, -4, -5


class EngineError(RuntimeError):
    pass


def load_library(path: str = LIB_PATH):
    """Loads libkp.so and declares the C-ABI signatures. Raises if it is absent."""
    if path in _LIBS:
        return _LIBS[path]
    if not os.path.exists(path):
        raise EngineError(f"{path} is missing: build it with `make -C karmada_amd/csrc` "
                          "(there is no CPU fallback)")
    L = C.CDLL(path)
    vp = C.c_void_p
    L.kp_abi_version.restype = C.c_int
    L.kp_engine_create.argtypes = [C.c_int, C.POINTER(vp)]
    L.kp_engine_destroy.argtypes = [vp]
    L.kp_last_error.restype = C.c_char_p
    L.kp_last_error.argtypes = [vp]
    L.kp_snapshot_create.argtypes = [vp, C.POINTER(api.kp_cluster), C.c_uint64, C.POINTER(api.kp_options),
                                     C.POINTER(vp)]
    L.kp_snapshot_destroy.argtypes = [vp]
    L.kp_batch_create.argtypes = [vp, vp, C.POINTER(api.kp_binding), C.c_uint64, C.POINTER(vp)]
    L.kp_batch_destroy.argtypes = [vp]
    L.kp_batch_digest.argtypes = [vp, C.POINTER(C.c_uint64)]
    L.kp_pack_cache_create.argtypes = [C.c_uint64, C.POINTER(vp)]
    L.kp_pack_cache_destroy.argtypes = [vp]
    L.kp_pack_cache_get_stats.argtypes = [vp, C.POINTER(api.kp_pack_cache_stats)]
    L.kp_batch_create_keyed.argtypes = [vp, vp, C.POINTER(api.kp_binding), C.POINTER(api.kp_binding_key), C.c_uint64,
                                        vp, C.POINTER(vp)]
    L.kp_schedule_batch.argtypes = [vp, vp, C.POINTER(api.kp_results)]
    L.kp_schedule_batch_submit.argtypes = [vp, vp]
    L.kp_schedule_batch_collect.argtypes = [vp, vp, C.POINTER(api.kp_results)]
    L.kp_schedule_affinities.argtypes = [vp, vp, C.POINTER(api.kp_binding), C.c_uint64,
                                         C.POINTER(api.kp_affinity_results)]
    L.kp_filter_batch.argtypes = [vp, vp, C.POINTER(C.c_uint64)]
    L.kp_score_batch.argtypes = [vp, vp, C.POINTER(C.c_int64)]
    L.kp_filter_reasons.argtypes = [vp, vp, C.POINTER(C.c_uint32)]
    L.kp_max_available_replicas.argtypes = [vp, vp, C.c_uint64, C.POINTER(C.c_uint32), C.c_uint64,
                                            C.POINTER(C.c_int32)]
    L.kp_max_available_component_sets.argtypes = [vp, vp, C.POINTER(api.kp_component), C.c_uint32,
                                                  C.POINTER(C.c_uint32), C.c_uint64, C.POINTER(C.c_int32)]
    L.kp_last_stage_times.argtypes = [vp, C.POINTER(api.kp_stage_times)]
    L.kp_model_grades.argtypes = [vp, C.POINTER(api.kp_resource_model), C.c_uint32, C.POINTER(api.kp_node),
                                  C.c_uint64, C.POINTER(C.c_int64)]
    L.kp_node_max_replicas.argtypes = [vp, C.POINTER(api.kp_node), C.c_uint64, C.POINTER(api.kp_resource), C.c_uint32,
                                       C.POINTER(api.kp_node_claim), C.POINTER(api.kp_assumed_workload), C.c_uint32,
                                       C.POINTER(C.c_int32)]
    L.kp_node_max_component_sets.argtypes = [vp, C.POINTER(api.kp_node), C.c_uint64, C.POINTER(api.kp_node_component),
                                             C.c_uint32, C.POINTER(api.kp_assumed_workload), C.c_uint32,
                                             C.POINTER(C.c_int32)]
    L.kp_snapshot_export.argtypes = [vp, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64)]
    L.kp_snapshot_import.argtypes = [vp, C.c_char_p, C.c_uint64, C.POINTER(vp)]
    L.kp_snapshot_update.argtypes = [vp, vp, C.POINTER(api.kp_cluster), C.c_uint64, C.POINTER(C.c_int)]
    L.kp_engine_set_threads.argtypes = [vp, C.c_int]
    L.kp_engine_set_profile.argtypes = [vp, C.c_int]
    L.kp_last_kernel_times.argtypes = [vp, C.POINTER(api.kp_kernel_time), C.c_uint32, C.POINTER(C.c_uint32)]
    L.kp_snapshot_replicate.argtypes = [vp, vp, C.POINTER(vp)]
    L.kp_multi_create.argtypes = [C.POINTER(C.c_int), C.c_uint32, C.POINTER(vp)]
    L.kp_multi_destroy.argtypes = [vp]
    L.kp_multi_last_error.restype = C.c_char_p
    L.kp_multi_last_error.argtypes = [vp]
    L.kp_multi_devices.restype = C.c_uint32
    L.kp_multi_devices.argtypes = [vp]
    L.kp_multi_engine.restype = vp
    L.kp_multi_engine.argtypes = [vp, C.c_uint32]
    L.kp_multi_snapshot_create.argtypes = [vp, C.POINTER(api.kp_cluster), C.c_uint64, C.POINTER(api.kp_options),
                                           C.POINTER(vp)]
    L.kp_multi_snapshot_update.argtypes = [vp, vp, C.POINTER(api.kp_cluster), C.c_uint64, C.POINTER(C.c_int)]
    L.kp_multi_snapshot_destroy.argtypes = [vp]
    L.kp_multi_snapshot_replica.restype = vp
    L.kp_multi_snapshot_replica.argtypes = [vp, C.c_uint32]
    L.kp_multi_shard_cuts.argtypes = [C.POINTER(api.kp_binding), C.c_uint64, C.c_uint64, C.c_uint32,
                                      C.POINTER(C.c_uint64)]
    L.kp_multi_batch_create.argtypes = [vp, vp, C.POINTER(api.kp_binding), C.c_uint64, C.POINTER(vp)]
    L.kp_multi_batch_destroy.argtypes = [vp]
    L.kp_multi_batch_shards.argtypes = [vp, C.POINTER(C.c_uint64)]
    L.kp_multi_schedule.argtypes = [vp, vp, C.POINTER(api.kp_results)]
    if L.kp_abi_version() != KP_ABI_VERSION:
        raise EngineError("libkp.so ABI version mismatch")
    _LIBS[path] = L
    return L


@dataclass
class TargetCluster:
    """workv1alpha2.TargetCluster (pkg/apis/work/v1alpha2/binding_types.go)."""
    name: str
    replicas: int


@dataclass
class ScheduleResult:
    """core.ScheduleResult (generic_scheduler.go:54-56) plus the error the reference returns."""
    suggested_clusters: List[TargetCluster] = field(default_factory=list)
    status: int = api.STATUS_OK
    err: int = 0
    arg: int = 0
    observed_affinity_name: Optional[str] = None  # set by schedule_with_affinities

    @property
    def error(self) -> Optional[str]:
        if self.status == api.STATUS_OK:
            return None
        return f"{api.ERR_NAMES.get(self.err, self.err)} ({self.arg})"


class Engine:
    """One HIP device + stream (kp_engine)."""

    def __init__(self, device: int = 0, lib_path: str = LIB_PATH):
        self.L = load_library(lib_path)
        h = C.c_void_p()
        rc = self.L.kp_engine_create(device, C.byref(h))
        if rc != KP_OK:
            raise EngineError(f"kp_engine_create(device={device}) failed: rc={rc}")
        self.h = h

    def _check(self, rc: int, what: str):
        if rc != KP_OK:
            raise EngineError(f"{what}: rc={rc}: {self.L.kp_last_error(self.h).decode(errors='replace')}")

    def close(self):
        if self.h:
            self.L.kp_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def model_grades(self, models: Sequence[dict], nodes: Sequence[dict]) -> List[int]:
        """getAllocatableModelings' AllocatableModeling counts, one per model
        (kp_model_grades; cluster_status_controller.go:642-677)."""
        w = api.World()
        ma, nm = w.models(models)
        na, nn = w.nodes(nodes)
        out = (C.c_int64 * max(1, nm))()
        self._check(self.L.kp_model_grades(self.h, ma, nm, na, nn, out), "kp_model_grades")
        return [int(out[i]) for i in range(nm)]

    def node_max_replicas(self, nodes: Sequence[dict], request: Optional[Dict[str, str]],
                          node_claim: Optional[dict] = None, assumed: Optional[Sequence[dict]] = None) -> int:
        """The estimator server's per-node answer (kp_node_max_replicas;
        noderesource.go:70-131) for one ReplicaRequirements, after the assumed
        workloads' deduction."""
        w = api.World()
        na, nn = w.nodes(nodes)
        ra, nr = w.resources(request)
        claim = w.node_claim(node_claim)
        aa, namd = w.assumed_workloads(assumed)
        out = C.c_int32()
        self._check(self.L.kp_node_max_replicas(self.h, na, nn, ra, nr, C.byref(claim) if claim is not None else None,
                                                aa, namd, C.byref(out)), "kp_node_max_replicas")
        return int(out.value)

    def node_max_component_sets(self, nodes: Sequence[dict], components: Sequence[dict],
                                assumed: Optional[Sequence[dict]] = None) -> int:
        """The estimator server's component-set answer (kp_node_max_component_sets;
        noderesource.go:146-190): complete sets of `components` the nodes hold."""
        w = api.World()
        na, nn = w.nodes(nodes)
        ca, nc = w.node_components(components)
        aa, namd = w.assumed_workloads(assumed)
        out = C.c_int32()
        self._check(self.L.kp_node_max_component_sets(self.h, na, nn, ca, nc, aa, namd, C.byref(out)),
                    "kp_node_max_component_sets")
        return int(out.value)

    def stage_times(self) -> Dict[str, float]:
        t = api.kp_stage_times()
        self._check(self.L.kp_last_stage_times(self.h, C.byref(t)), "kp_last_stage_times")
        return {k: getattr(t, k) for k, _ in api.kp_stage_times._fields_}

    def set_profile(self, on: bool = True):
        """Per-kernel HIP-event timing of kp_schedule_batch (kp_engine_set_profile)."""
        self._check(self.L.kp_engine_set_profile(self.h, int(on)), "kp_engine_set_profile")

    def kernel_times(self) -> Dict[str, dict]:
        """{kernel name: {ms, launches, units}} of the last kp_schedule_batch (profiling on)."""
        n = C.c_uint32()
        self._check(self.L.kp_last_kernel_times(self.h, None, 0, C.byref(n)), "kp_last_kernel_times")
        arr = (api.kp_kernel_time * max(1, n.value))()
        self._check(self.L.kp_last_kernel_times(self.h, arr, n.value, C.byref(n)), "kp_last_kernel_times")
        return {arr[i].name.decode(): {"ms": arr[i].ms, "launches": arr[i].launches, "units": arr[i].units}
                for i in range(n.value)}


class Snapshot:
    """cache.Snapshot (pkg/scheduler/cache/snapshot.go) packed into HBM."""

    def __init__(self, engine: Engine, clusters: Sequence[dict], opts: Optional[api.kp_options] = None):
        self.engine = engine
        self.names = [c["name"] for c in clusters]
        w = api.World()
        ca, n = w.clusters(clusters)
        self.opts = opts or api.options()
        h = C.c_void_p()
        engine._check(engine.L.kp_snapshot_create(engine.h, ca, n, C.byref(self.opts), C.byref(h)),
                      "kp_snapshot_create")
        self.h = h

    @classmethod
    def from_structs(cls, engine: Engine, ca, n: int, names: List[str], opts: api.kp_options):
        self = cls.__new__(cls)
        self.engine, self.names, self.opts = engine, names, opts
        h = C.c_void_p()
        engine._check(engine.L.kp_snapshot_create(engine.h, ca, n, C.byref(opts), C.byref(h)), "kp_snapshot_create")
        self.h = h
        return self

    def to_bytes(self) -> bytes:
        """Packed snapshot bytes (kp_snapshot_export) for broadcast to other ranks."""
        p, n = C.c_void_p(), C.c_uint64()
        self.engine._check(self.engine.L.kp_snapshot_export(self.h, C.byref(p), C.byref(n)), "kp_snapshot_export")
        return C.string_at(p, n.value)

    @classmethod
    def from_bytes(cls, engine: Engine, data: bytes, names: List[str]):
        """kp_snapshot_import: the packed snapshot of another rank, uploaded to this engine's device."""
        self = cls.__new__(cls)
        self.engine, self.names, self.opts = engine, names, None
        h = C.c_void_p()
        engine._check(engine.L.kp_snapshot_import(engine.h, data, len(data), C.byref(h)), "kp_snapshot_import")
        self.h = h
        return self

    def update_structs(self, ca, n: int) -> bool:
        """kp_snapshot_update: re-pack the n clusters of `ca` (existing names) in place.
        Returns True when the dictionaries grew (batches packed before must be re-created)."""
        grew = C.c_int(0)
        self.engine._check(self.engine.L.kp_snapshot_update(self.engine.h, self.h, ca, n, C.byref(grew)),
                           "kp_snapshot_update")
        return bool(grew.value)

    def update(self, clusters: Sequence[dict]) -> bool:
        """Cluster events (informer updates) applied to the packed snapshot; see update_structs."""
        w = api.World()
        ca, n = w.clusters(clusters)
        return self.update_structs(ca, n)

    def close(self):
        if getattr(self, "h", None):
            self.engine.L.kp_snapshot_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PackCache:
    """Packed binding records kept across scheduling cycles (kp_pack_cache): a binding
    whose (metadata.uid, metadata.generation) and scheduler status fields match a record
    is copied instead of re-packed (pkg/scheduler/scheduler.go:437-468 re-runs Schedule
    for bindings whose spec did not change)."""

    def __init__(self, engine: "Engine", max_entries: int = 0):
        self.L = engine.L
        h = C.c_void_p()
        if self.L.kp_pack_cache_create(max_entries, C.byref(h)) != KP_OK:
            raise EngineError("kp_pack_cache_create failed")
        self.h = h

    def stats(self) -> dict:
        st = api.kp_pack_cache_stats()
        self.L.kp_pack_cache_get_stats(self.h, C.byref(st))
        return {"hits": st.hits, "misses": st.misses, "entries": st.entries, "last_hits": st.last_hits}

    def close(self):
        if getattr(self, "h", None):
            self.L.kp_pack_cache_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Batch:
    """A batch of ResourceBindings packed against one snapshot (kp_batch). With `cache`
    and `keys` ((uid, generation) per binding, api.binding_keys) it is created through
    kp_batch_create_keyed: bindings whose record the cache holds skip packing."""

    def __init__(self, snap: Snapshot, bindings: Sequence[dict] = (), structs=None, cache: "PackCache" = None,
                 keys=None, generations: Sequence[int] = None):
        self.snap = snap
        eng = snap.engine
        if structs is None:
            w = api.World()
            ba, n = w.bindings(bindings)
            self._w = w
        else:
            ba, n = structs
        self.n = n
        h = C.c_void_p()
        if cache is not None:
            if keys is None:  # (uid from each binding, metadata.generation given)
                keys = api.binding_keys(ba, n, generations if generations is not None else [0] * n)
            self._keys = keys
            eng._check(eng.L.kp_batch_create_keyed(eng.h, snap.h, ba, keys, n, cache.h, C.byref(h)),
                       "kp_batch_create_keyed")
        else:
            eng._check(eng.L.kp_batch_create(eng.h, snap.h, ba, n, C.byref(h)), "kp_batch_create")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.snap.engine.L.kp_batch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def digest(self) -> int:
        """kp_batch_digest: the packed image's digest (equal for equal packs)."""
        d = C.c_uint64()
        self.snap.engine._check(self.snap.engine.L.kp_batch_digest(self.h, C.byref(d)), "kp_batch_digest")
        return d.value

    def schedule_raw(self) -> api.kp_results:
        r = api.kp_results()
        eng = self.snap.engine
        eng._check(eng.L.kp_schedule_batch(eng.h, self.h, C.byref(r)), "kp_schedule_batch")
        return r

    def submit(self):
        """kp_schedule_batch_submit: queue this batch's schedule call (collect() finishes it)."""
        eng = self.snap.engine
        eng._check(eng.L.kp_schedule_batch_submit(eng.h, self.h), "kp_schedule_batch_submit")

    def collect(self) -> api.kp_results:
        """kp_schedule_batch_collect: the results of the submitted call (as schedule_raw)."""
        r = api.kp_results()
        eng = self.snap.engine
        eng._check(eng.L.kp_schedule_batch_collect(eng.h, self.h, C.byref(r)), "kp_schedule_batch_collect")
        return r

    def schedule(self) -> List[dict]:
        """Results as api.results_to_python dicts (cluster indices in snapshot input order)."""
        r = self.schedule_raw()
        return api.results_to_python(r.status, r.err_code, r.err_arg, r.offsets, r.cluster_idx, r.replicas,
                                     r.n_bindings)


class MultiEngine:
    """One scheduler process over N GPUs (kp_multi): an engine per device, the snapshot
    replicated device to device, each batch sharded by cost across the devices and
    scheduled concurrently, results merged in binding order. Replaces the reference
    scheduler's single worker (pkg/scheduler/scheduler.go:327)."""

    def __init__(self, devices: Sequence[int], lib_path: str = LIB_PATH):
        self.L = load_library(lib_path)
        devs = (C.c_int * len(devices))(*devices)
        h = C.c_void_p()
        rc = self.L.kp_multi_create(devs, len(devices), C.byref(h))
        if rc != KP_OK:
            raise EngineError(f"kp_multi_create(devices={list(devices)}) failed: rc={rc}")
        self.h = h
        self.n_devices = int(self.L.kp_multi_devices(h))

    def _check(self, rc: int, what: str):
        if rc != KP_OK:
            raise EngineError(f"{what}: rc={rc}: {self.L.kp_multi_last_error(self.h).decode(errors='replace')}")

    def stage_times(self, i: int) -> Dict[str, float]:
        """kp_last_stage_times of device i's engine (its shard's last schedule)."""
        t = api.kp_stage_times()
        e = self.L.kp_multi_engine(self.h, i)
        if self.L.kp_last_stage_times(e, C.byref(t)) != KP_OK:
            raise EngineError("kp_last_stage_times")
        return {k: getattr(t, k) for k, _ in api.kp_stage_times._fields_}

    def snapshot(self, ca, n: int, opts: api.kp_options) -> "MultiSnapshot":
        return MultiSnapshot(self, ca, n, opts)

    def close(self):
        if getattr(self, "h", None):
            self.L.kp_multi_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MultiSnapshot:
    """kp_multi_snapshot: packed on the first device, replicas on the others."""

    def __init__(self, m: MultiEngine, ca, n: int, opts: api.kp_options):
        self.m, self.opts, self.n_clusters = m, opts, n
        h = C.c_void_p()
        m._check(m.L.kp_multi_snapshot_create(m.h, ca, n, C.byref(opts), C.byref(h)), "kp_multi_snapshot_create")
        self.h = h

    def update_structs(self, ca, n: int) -> bool:
        grew = C.c_int(0)
        self.m._check(self.m.L.kp_multi_snapshot_update(self.m.h, self.h, ca, n, C.byref(grew)),
                      "kp_multi_snapshot_update")
        return bool(grew.value)

    def close(self):
        if getattr(self, "h", None):
            self.m.L.kp_multi_snapshot_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MultiBatch:
    """kp_multi_batch: a batch cut into per-device shards."""

    def __init__(self, snap: MultiSnapshot, structs):
        self.snap = snap
        m = snap.m
        ba, n = structs
        self.n = n
        h = C.c_void_p()
        m._check(m.L.kp_multi_batch_create(m.h, snap.h, ba, n, C.byref(h)), "kp_multi_batch_create")
        self.h = h

    def shards(self) -> List[int]:
        D = self.snap.m.n_devices
        out = (C.c_uint64 * (D + 1))()
        self.snap.m._check(self.snap.m.L.kp_multi_batch_shards(self.h, out), "kp_multi_batch_shards")
        return [int(out[i]) for i in range(D + 1)]

    def schedule_raw(self) -> api.kp_results:
        r = api.kp_results()
        m = self.snap.m
        m._check(m.L.kp_multi_schedule(m.h, self.h, C.byref(r)), "kp_multi_schedule")
        return r

    def schedule(self) -> List[dict]:
        r = self.schedule_raw()
        return api.results_to_python(r.status, r.err_code, r.err_arg, r.offsets, r.cluster_idx, r.replicas,
                                     r.n_bindings)

    def close(self):
        if getattr(self, "h", None):
            self.snap.m.L.kp_multi_batch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class GenericScheduler:
    """genericScheduler (generic_scheduler.go:38-121) over a snapshot, batched."""

    def __init__(self, engine: Engine, clusters: Sequence[dict], opts: Optional[api.kp_options] = None):
        self.snapshot = Snapshot(engine, clusters, opts)

    def schedule(self, bindings: Sequence[dict]) -> List[ScheduleResult]:
        b = Batch(self.snapshot, bindings)
        out = []
        names = self.snapshot.names
        for r in b.schedule():
            sr = ScheduleResult(status=r["status"], err=r["err"], arg=r["arg"])
            sr.suggested_clusters = [TargetCluster(names[i], rep) for i, rep in r["targets"]]
            out.append(sr)
        b.close()
        return out

    def schedule_affinities_raw(self, structs):
        """kp_schedule_affinities over packed kp_binding structs: (results dicts, affinity_index, attempts, rounds)."""
        ba, n = structs
        eng = self.snapshot.engine
        r = api.kp_affinity_results()
        eng._check(eng.L.kp_schedule_affinities(eng.h, self.snapshot.h, ba, n, C.byref(r)), "kp_schedule_affinities")
        rr = r.results
        res = api.results_to_python(rr.status, rr.err_code, rr.err_arg, rr.offsets, rr.cluster_idx, rr.replicas,
                                    rr.n_bindings)
        return res, [int(r.affinity_index[i]) for i in range(n)], [int(r.attempts[i]) for i in range(n)], r.rounds

    def schedule_with_affinities(self, bindings: Sequence[dict]) -> List[ScheduleResult]:
        """Scheduler.scheduleResourceBindingWithClusterAffinities (scheduler.go:618-684) per binding,
        batched: every term retry of a round runs as one device batch. Each result carries the
        AffinityName that became Status.SchedulerObservedAffinityName (None: unchanged)."""
        w = api.World()
        structs = w.bindings(bindings)
        res, aff, _, _ = self.schedule_affinities_raw(structs)
        names = self.snapshot.names
        out = []
        for b, r, a in zip(bindings, res, aff):
            sr = ScheduleResult(status=r["status"], err=r["err"], arg=r["arg"])
            sr.suggested_clusters = [TargetCluster(names[i], rep) for i, rep in r["targets"]]
            terms = (b.get("placement") or {}).get("clusterAffinities") or []
            sr.observed_affinity_name = terms[a].get("affinityName") if a >= 0 else None
            out.append(sr)
        return out

    def filter(self, bindings: Sequence[dict]) -> List[List[str]]:
        """Feasible cluster names per binding (findClustersThatFit)."""
        b = Batch(self.snapshot, bindings)
        eng = self.snapshot.engine
        C_ = len(self.snapshot.names)
        W = (C_ + 63) // 64
        m = (C.c_uint64 * max(1, b.n * W))()
        eng._check(eng.L.kp_filter_batch(eng.h, b.h, m), "kp_filter_batch")
        out = []
        for i in range(b.n):
            out.append([self.snapshot.names[c] for c in range(C_) if (m[i * W + (c >> 6)] >> (c & 63)) & 1])
        b.close()
        return out

    def filter_reasons(self, bindings: Sequence[dict]) -> List[List[int]]:
        """kp_filter_reasons: the KP_REASON_* word of every (binding, cluster) pair."""
        b = Batch(self.snapshot, bindings)
        eng = self.snapshot.engine
        C_ = len(self.snapshot.names)
        r = (C.c_uint32 * max(1, b.n * C_))()
        eng._check(eng.L.kp_filter_reasons(eng.h, b.h, r), "kp_filter_reasons")
        out = [[int(r[i * C_ + c]) for c in range(C_)] for i in range(b.n)]
        b.close()
        return out

    def fit_error(self, binding: dict, clusters: Sequence[dict]) -> str:
        """FitError{NumAllClusters, Diagnosis}.Error() for one binding (generic_scheduler.go:84-89);
        `clusters` are the snapshot's cluster dicts in its caller order."""
        codes = self.filter_reasons([binding])[0]
        reasons = {cl["name"]: api.reason_text(code, cl) for cl, code in zip(clusters, codes)
                   if code not in (api.REASON_FIT, api.REASON_DELETING)}
        return api.fit_error_message(len(clusters), reasons)

    def score(self, bindings: Sequence[dict]) -> List[List[int]]:
        """Summed plugin scores per (binding, cluster) (prioritizeClusters)."""
        b = Batch(self.snapshot, bindings)
        eng = self.snapshot.engine
        C_ = len(self.snapshot.names)
        s = (C.c_int64 * max(1, b.n * C_))()
        eng._check(eng.L.kp_score_batch(eng.h, b.h, s), "kp_score_batch")
        out = [[int(s[i * C_ + c]) for c in range(C_)] for i in range(b.n)]
        b.close()
        return out

    def max_available_component_sets(self, components: Sequence[dict], clusters: Sequence[str]) -> List[int]:
        """GeneralEstimator.MaxAvailableComponentSets (general.go:154-162) for one
        component list; raises EngineError (KP_ENOTSUP) with the gate off."""
        eng = self.snapshot.engine
        w = api.World()
        ca, nc = w.components(components)
        idx = {n: i for i, n in enumerate(self.snapshot.names)}
        ci = (C.c_uint32 * max(1, len(clusters)))(*[idx[n] for n in clusters])
        out = (C.c_int32 * max(1, len(clusters)))()
        eng._check(eng.L.kp_max_available_component_sets(eng.h, self.snapshot.h, ca, nc, ci, len(clusters), out),
                   "kp_max_available_component_sets")
        return [int(out[i]) for i in range(len(clusters))]

    def max_available_replicas(self, binding: dict, clusters: Sequence[str]) -> List[int]:
        """GeneralEstimator.MaxAvailableReplicas for one binding's request."""
        b = Batch(self.snapshot, [binding])
        eng = self.snapshot.engine
        idx = {n: i for i, n in enumerate(self.snapshot.names)}
        ci = (C.c_uint32 * max(1, len(clusters)))(*[idx[n] for n in clusters])
        out = (C.c_int32 * max(1, len(clusters)))()
        eng._check(eng.L.kp_max_available_replicas(eng.h, b.h, 0, ci, len(clusters), out),
                   "kp_max_available_replicas")
        b.close()
        return [int(out[i]) for i in range(len(clusters))]
