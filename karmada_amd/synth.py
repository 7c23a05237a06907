"""Seeded synthetic Karmada universes (csrc/synth.cpp) as kp_api.h structs."""
from __future__ import annotations

import ctypes as C
import os

from karmada_amd import api

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG, "libkpsynth.so")
_LIB = None

# BASELINE.json configs: (clusters, bindings)
CONFIGS = {
    1: (10, 1_000),
    2: (1_000, 100_000),
    3: (5_000, 100_000),
    4: (5_000, 100_000),
    5: (10_000, 1_000_000),
    6: (300, 5_000),   # edge workload (every branch), parity only
    7: (2_000, 5_000),  # Aggregated tie straddles (sort.Sort permutation), parity only
    8: (64, 2_000),     # int32 wrap of replica sums, weights >= 2^31, parity only
    9: (2_000, 5_000),  # multi-template workloads (MultiplePodTemplatesScheduling), parity only
    10: (5_000, 100_000),  # config 3 with per-binding-distinct requests (estimator classes ~ bindings)
    11: (5_000, 5_000),  # spread constraints with MinGroups 0, parity only
}


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make -C karmada_amd/csrc`")
        L = C.CDLL(LIB_PATH)
        L.kps_create.argtypes = [C.c_int, C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint64, C.POINTER(C.c_void_p)]
        L.kps_destroy.argtypes = [C.c_void_p]
        L.kps_clusters.restype = C.POINTER(api.kp_cluster)
        L.kps_clusters.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
        L.kps_bindings.restype = C.POINTER(api.kp_binding)
        L.kps_bindings.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
        L.kps_replicas.argtypes = [C.c_int, C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint64, C.POINTER(C.c_int32)]
        _LIB = L
    return _LIB


def replicas(config: int, seed: int, n_clusters: int, lo: int, hi: int):
    """spec.Replicas of bindings [lo, hi) of the universe (numpy int32), for shard costs."""
    import numpy as np
    out = np.zeros(max(0, hi - lo), dtype=np.int32)
    if len(out) and lib().kps_replicas(config, seed, n_clusters, lo, hi,
                                        out.ctypes.data_as(C.POINTER(C.c_int32))) != 0:
        raise RuntimeError("kps_replicas failed")
    return out


class Universe:
    """Clusters [0, C) and bindings [lo, hi) of workload `config` with `seed`."""

    def __init__(self, config: int, seed: int, n_clusters: int, lo: int, hi: int):
        L = lib()
        h = C.c_void_p()
        if L.kps_create(config, seed, n_clusters, lo, hi, C.byref(h)) != 0:
            raise RuntimeError("kps_create failed")
        self.h = h
        n = C.c_uint64()
        self.clusters = L.kps_clusters(h, C.byref(n))
        self.n_clusters = n.value
        self.bindings = L.kps_bindings(h, C.byref(n))
        self.n_bindings = n.value
        self.names = [f"member-{i:05d}" if n_clusters <= 99999 else f"member-{i:07d}" for i in range(n_clusters)]

    def binding_slice(self, lo: int, hi: int):
        """(pointer, count) of bindings [lo, hi) relative to this universe's range."""
        base = C.cast(self.bindings, C.c_void_p).value + lo * C.sizeof(api.kp_binding)
        return C.cast(C.c_void_p(base), C.POINTER(api.kp_binding)), hi - lo

    def close(self):
        if getattr(self, "h", None):
            lib().kps_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
