"""Loads the CPU oracle (oracle/liboracle.so) for tests. Test infrastructure only."""
import ctypes as C
import os
import subprocess

from karmada_amd import api

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
_LIB = None


class kpo_results(C.Structure):
    _fields_ = [("n", C.c_uint64), ("status", C.POINTER(C.c_int32)), ("err_code", C.POINTER(C.c_int32)),
                ("err_arg", C.POINTER(C.c_int64)), ("offsets", C.POINTER(C.c_uint64)),
                ("cluster_idx", C.POINTER(C.c_uint32)), ("replicas", C.POINTER(C.c_int32)),
                ("n_targets", C.c_uint64)]


class kpo_candidate(C.Structure):
    _fields_ = [("name", api.kp_str), ("score", C.c_int64), ("overflow_order", C.c_int32),
                ("available_replicas", C.c_int64), ("allocatable_replicas", C.c_int32), ("cluster", C.c_int32)]


def lib():
    global _LIB
    if _LIB is not None:
        return _LIB
    path = os.path.join(ORACLE_DIR, "liboracle.so")
    src = os.path.join(ORACLE_DIR, "oracle.cpp")
    if (not os.path.exists(path)) or os.path.getmtime(path) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
    L = C.CDLL(path)
    L.kpo_world_create.restype = C.c_void_p
    L.kpo_world_create.argtypes = [C.POINTER(api.kp_cluster), C.c_uint64, C.POINTER(api.kp_options)]
    L.kpo_world_destroy.argtypes = [C.c_void_p]
    L.kpo_schedule.argtypes = [C.c_void_p, C.POINTER(api.kp_binding), C.c_uint64, C.c_int, C.c_int,
                               C.POINTER(C.POINTER(kpo_results))]
    L.kpo_schedule_affinities.argtypes = [C.c_void_p, C.POINTER(api.kp_binding), C.c_uint64, C.c_int, C.c_int,
                                          C.POINTER(C.POINTER(kpo_results)), C.POINTER(C.c_int32),
                                          C.POINTER(C.c_int32)]
    L.kpo_results_free.argtypes = [C.POINTER(kpo_results)]
    L.kpo_quantity.argtypes = [C.c_char_p, C.c_uint32, C.c_int, C.POINTER(C.c_int64)]
    L.kpo_cluster_matches.argtypes = [C.POINTER(api.kp_cluster), C.POINTER(api.kp_cluster_affinity)]
    L.kpo_filter.restype = C.c_uint32
    L.kpo_filter.argtypes = [C.POINTER(api.kp_cluster), C.POINTER(api.kp_binding), C.POINTER(api.kp_options)]
    L.kpo_score.restype = C.c_int64
    L.kpo_score.argtypes = [C.POINTER(api.kp_cluster), C.POINTER(api.kp_binding), C.POINTER(api.kp_options)]
    L.kpo_max_available_replicas.restype = C.c_int32
    L.kpo_max_available_replicas.argtypes = [C.POINTER(api.kp_cluster), C.POINTER(api.kp_binding),
                                             C.POINTER(api.kp_options), C.c_int]
    L.kpo_allocate_webster.argtypes = [C.c_int32, C.POINTER(api.kp_str), C.POINTER(C.c_int64), C.c_uint32,
                                       C.POINTER(api.kp_str), C.POINTER(C.c_int32), C.c_uint32, C.c_int, api.kp_str,
                                       C.POINTER(C.c_int32), C.c_uint32]
    L.kpo_spread_replicas.argtypes = [C.c_int32, C.POINTER(api.kp_target_cluster), C.c_uint32,
                                      C.POINTER(api.kp_target_cluster), C.c_uint32, api.kp_str,
                                      C.POINTER(api.kp_target_cluster), C.c_uint32]
    L.kpo_assign_replicas.argtypes = [C.POINTER(kpo_candidate), C.c_uint32, C.POINTER(api.kp_cluster), C.c_uint32,
                                      C.POINTER(api.kp_binding), C.c_int, C.POINTER(C.c_int32),
                                      C.POINTER(C.c_int64), C.POINTER(api.kp_target_cluster), C.c_uint32]
    L.kpo_select_groups.argtypes = [C.POINTER(api.kp_str), C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.c_uint32,
                                    C.c_int64, C.c_int64, C.c_int64, C.POINTER(C.c_uint32)]
    L.kpo_calc_group_score.restype = C.c_int64
    L.kpo_h4_hits.restype = C.c_uint64
    L.kpo_h4_hits.argtypes = [C.c_int]
    L.kpo_calc_group_score.argtypes = [C.POINTER(kpo_candidate), C.c_uint32, C.POINTER(api.kp_binding), C.c_int64]
    L.kpo_select_clusters.argtypes = [C.POINTER(api.kp_cluster), C.POINTER(C.c_int64), C.POINTER(C.c_int32),
                                      C.c_uint32, C.POINTER(api.kp_binding), C.c_int32, C.POINTER(C.c_uint32),
                                      C.c_uint32]
    L.kpo_sort_target_clusters.argtypes = [C.POINTER(C.c_int32), C.POINTER(C.c_uint32), C.c_uint32]
    L.kpo_fnv32a.restype = C.c_uint32
    L.kpo_fnv32a.argtypes = [C.c_char_p, C.c_uint32]
    _LIB = L
    return L


FAITHFUL, FAST, REFSHAPE = 0, 1, 2


def schedule(clusters, bindings, opts=None, mode=FAITHFUL, threads=1):
    """Runs the oracle over dict inputs; returns api.results_to_python list."""
    w = api.World()
    ca, nc = w.clusters(clusters)
    ba, nb = w.bindings(bindings)
    o = opts or api.options()
    return schedule_c(ca, nc, ba, nb, o, mode, threads)


def schedule_c(ca, nc, ba, nb, opts, mode=FAITHFUL, threads=1):
    L = lib()
    world = L.kpo_world_create(ca, nc, C.byref(opts))
    try:
        rp = C.POINTER(kpo_results)()
        L.kpo_schedule(world, ba, nb, mode, threads, C.byref(rp))
        r = rp.contents
        out = api.results_to_python(r.status, r.err_code, r.err_arg, r.offsets, r.cluster_idx, r.replicas, r.n)
        L.kpo_results_free(rp)
        return out
    finally:
        L.kpo_world_destroy(world)


def schedule_affinities_c(ca, nc, ba, nb, opts, mode=FAITHFUL, threads=1):
    """scheduleResourceBindingWithClusterAffinities per binding: (results, affinity_index, attempts)."""
    L = lib()
    world = L.kpo_world_create(ca, nc, C.byref(opts))
    try:
        rp = C.POINTER(kpo_results)()
        aff = (C.c_int32 * max(1, nb))()
        att = (C.c_int32 * max(1, nb))()
        L.kpo_schedule_affinities(world, ba, nb, mode, threads, C.byref(rp), aff, att)
        r = rp.contents
        out = api.results_to_python(r.status, r.err_code, r.err_arg, r.offsets, r.cluster_idx, r.replicas, r.n)
        L.kpo_results_free(rp)
        return out, list(aff[:nb]), list(att[:nb])
    finally:
        L.kpo_world_destroy(world)
