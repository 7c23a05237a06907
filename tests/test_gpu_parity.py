"""GPU parity: libkp.so (HIP, gfx950) against the CPU oracle on seeded universes.

Bit-exact bar: status, error code and argument, and the multiset of
(cluster, replicas) targets per binding (IsScheduleResultEqual semantics:
reference pkg/scheduler/core/generic_scheduler_test.go compares sorted
TargetClusters). The oracle's fast mode is itself pinned to its faithful mode
in tests/test_oracle_synth.py and to the reference golden vectors in
tests/test_oracle_golden.py.
"""
import ctypes as C

import pytest

from karmada_amd import api, synth
import oracle_lib as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    from karmada_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


def gpu_schedule(engine, u, opts, lo=0, hi=None):
    from karmada_amd.engine import Batch, Snapshot
    hi = u.n_bindings if hi is None else hi
    snap = Snapshot.from_structs(engine, u.clusters, u.n_clusters, u.names, opts)
    b = Batch(snap, structs=u.binding_slice(lo, hi))
    out = b.schedule()
    b.close()
    snap.close()
    return out


def oracle_schedule(u, opts, lo=0, hi=None):
    hi = u.n_bindings if hi is None else hi
    ba, n = u.binding_slice(lo, hi)
    return O.schedule_c(u.clusters, u.n_clusters, ba, n, opts, O.FAST, 8)


def compare(got, want, label):
    assert len(got) == len(want)
    bad = [i for i, (g, w) in enumerate(zip(got, want)) if g != w]
    if bad:
        lines = [f"{label}: {len(bad)}/{len(want)} bindings differ"]
        for i in bad[:5]:
            lines.append(f"  binding {i}: gpu={got[i]}")
            lines.append(f"  binding {i}: ref={want[i]}")
        pytest.fail("\n".join(lines))


CASES = [
    # (config, seed, clusters, bindings)
    (1, 1, 10, 1000),
    (2, 2, 1000, 2000),
    (3, 3, 500, 1000),
    (4, 4, 1000, 2000),
    (6, 6, 300, 3000),
    (6, 7, 64, 3000),
    (6, 8, 1, 500),
    (6, 9, 700, 2000),
    # Aggregated ties straddling the cut at every list length: k_slow's
    # sort.Sort wave emulation + block-parallel cut (kp_pdq.h)
    (7, 17, 2000, 3000),
    (7, 18, 13, 2000),
    (7, 19, 100, 2000),
    (7, 20, 5000, 1000),
    # overflow tiers with ~5k-entry serial lists in many concurrent k_slow workgroups
    # (the serial scratch sizing fix)
    (6, 13, 5000, 4000),
    # C > ~8.6k: gathered candidates would leave one workgroup per CU, so in the
    # bitset mode the SEL_ALL bindings take k_select_all_stream (the pair-row test
    # below runs the gathered k_select_all_wide at this size)
    (6, 21, 9000, 1000),
    (7, 22, 9000, 600),
    # int32 wrap of replica sums, StaticWeight weights >= 2^31 and seat counts past
    # 2^30 (SURVEY hazard H5): k_slow's serial route (SLOW_WRAP / SLOW_WEIGHT)
    (8, 4, 64, 2000),
    (8, 5, 16, 600),
    (8, 6, 300, 1500),
    # BASELINE configs at the cluster counts they are quoted on (binding slices of
    # the bench universes: same seeds as bench.py)
    (3, 3, 5000, 2000),
    (4, 4, 5000, 2000),
    (5, 5, 10000, 1500),
    (2, 2, 1000, 4000),
]


@pytest.mark.parametrize("config,seed,n_clusters,n_bindings", CASES)
def test_schedule_parity(engine, config, seed, n_clusters, n_bindings):
    u = synth.Universe(config, seed, n_clusters, 0, n_bindings)
    opts = api.options()
    compare(gpu_schedule(engine, u, opts), oracle_schedule(u, opts), f"config {config} seed {seed}")
    if config in (4, 5):  # cluster spread without spec.Clusters: the class-order selection ran
        t = engine.stage_times()
        assert 0 < t["n_cluster_order"] <= t["n_cluster"]
        if config == 4:
            assert 0 < t["n_region_order"] <= t["n_region"]


@pytest.mark.parametrize("config,seed,n_clusters,n_bindings", [
    (10, 10, 5000, 2000), (3, 3, 5000, 2000), (7, 17, 2000, 3000), (7, 18, 13, 2000), (6, 9, 700, 2000),
    (8, 4, 64, 2000), (8, 6, 300, 1500),
])
def test_schedule_parity_top_histogram(engine, config, seed, n_clusters, n_bindings):
    """k_select_top without class orders (config 10: about one estimator class per
    binding; the others forced with KP_ORDER_AMORT): the votes thresholded by an octave
    histogram instead of a walk of the class order (kp_top.h)."""
    import os
    u = synth.Universe(config, seed, n_clusters, 0, n_bindings)
    opts = api.options()
    os.environ["KP_ORDER_AMORT"] = "1000000"
    try:
        got = gpu_schedule(engine, u, opts)
        t = engine.stage_times()
    finally:
        os.environ.pop("KP_ORDER_AMORT", None)
    compare(got, oracle_schedule(u, opts), f"histogram config {config} seed {seed}")
    assert t["n_top"] > 0


@pytest.mark.parametrize("mid", ["64", "128"])
@pytest.mark.parametrize("config,seed,n_clusters,n_bindings", [
    (3, 3, 5000, 3000), (7, 17, 2000, 3000), (6, 9, 700, 2000), (10, 10, 5000, 2000),
])
def test_schedule_parity_top_mid_capacity(config, seed, n_clusters, n_bindings, mid):
    """k_select_top's large slice at a small first capacity (KP_TOP_CAP_MID): the bindings
    whose subset outgrows it are appended to the overflow list and run again at the full
    capacity by the grid-stride launch over that device list (engine.cpp), whose own
    overflow goes to the full-candidate kernel: the oracle's placements."""
    import os
    from karmada_amd.engine import Engine
    u = synth.Universe(config, seed, n_clusters, 0, n_bindings)
    opts = api.options()
    os.environ["KP_TOP_CAP_MID"] = mid  # (read at engine creation)
    try:
        e = Engine(0)
    finally:
        os.environ.pop("KP_TOP_CAP_MID", None)
    try:
        got = gpu_schedule(e, u, opts)
        t = e.stage_times()
    finally:
        e.close()
    compare(got, oracle_schedule(u, opts), f"mid capacity {mid} config {config} seed {seed}")
    assert t["n_top"] > 0


@pytest.mark.parametrize("config,seed,n_clusters,n_bindings", [
    (3, 3, 500, 1000), (2, 2, 1000, 1000), (5, 5, 3000, 1200), (7, 17, 2000, 1000), (3, 3, 5000, 1000),
    # C >= 9000: the gathered SEL_ALL kernel needs more than 80 KB of LDS -> k_select_all_wide
    (6, 21, 9000, 600), (7, 22, 9000, 400), (3, 23, 10000, 300),
])
def test_schedule_parity_pair_rows(engine, config, seed, n_clusters, n_bindings):
    """The per-binding pair-row route (KP_PAIR_ROWS=1: k_pair_fast_* writes every
    binding's feasibility and calAvailableReplicas rows) beside the default
    bitset filter + estimator classes."""
    import os
    u = synth.Universe(config, seed, n_clusters, 0, n_bindings)
    opts = api.options()
    os.environ["KP_PAIR_ROWS"] = "1"
    try:
        got = gpu_schedule(engine, u, opts)
        bits = engine.stage_times()["bits"]
    finally:
        os.environ.pop("KP_PAIR_ROWS", None)
    compare(got, oracle_schedule(u, opts), f"pair rows config {config} seed {seed}")
    assert bits == 0


@pytest.mark.parametrize("rows", [False, True], ids=["bits", "rows"])
@pytest.mark.parametrize("config,seed,n_clusters,n_bindings,multi", [
    (9, 31, 2000, 2000, True), (9, 32, 500, 1500, False), (6, 33, 300, 2000, True), (9, 34, 5000, 800, True),
])
def test_schedule_parity_multi_templates(engine, config, seed, n_clusters, n_bindings, multi, rows):
    """MultiplePodTemplatesScheduling: bindings that isMultiTemplateSchedulingApplicable
    accepts take MaxAvailableComponentSets as their estimator row (k_sets_rows; core/
    util.go:113-118, estimation.go:77-113) and need one replica in SelectBestClusters
    (common.go:42-46); with the gate off the same bindings take the single-template
    route."""
    import os
    u = synth.Universe(config, seed, n_clusters, 0, n_bindings)
    opts = api.options(multi_templates=multi)
    if rows:
        os.environ["KP_PAIR_ROWS"] = "1"
    try:
        got = gpu_schedule(engine, u, opts)
    finally:
        os.environ.pop("KP_PAIR_ROWS", None)
    compare(got, oracle_schedule(u, opts), f"multi-templates {multi} config {config} seed {seed}")


@pytest.mark.parametrize("prop,plugins,gate", [
    (True, api.PLUGIN_ALL, True),
    (False, api.PLUGIN_ALL & ~api.PLUGIN_TAINT_TOLERATION, True),
    (False, api.PLUGIN_ALL & ~api.PLUGIN_CLUSTER_LOCALITY, False),
    (False, 0, True),
])
def test_schedule_parity_options(engine, prop, plugins, gate):
    u = synth.Universe(6, 11, 200, 0, 1500)
    opts = api.options(empty_workload_propagation=prop, models_gate=gate, plugins=plugins)
    compare(gpu_schedule(engine, u, opts), oracle_schedule(u, opts), f"options {prop} {plugins} {gate}")


def test_filter_score_estimate_parity(engine):
    from karmada_amd.engine import Batch, Snapshot
    u = synth.Universe(6, 12, 130, 0, 300)
    opts = api.options()
    snap = Snapshot.from_structs(engine, u.clusters, u.n_clusters, u.names, opts)
    b = Batch(snap, structs=u.binding_slice(0, u.n_bindings))
    L = engine.L
    nC, nB = u.n_clusters, u.n_bindings
    W = (nC + 63) // 64
    mask = (C.c_uint64 * (nB * W))()
    engine._check(L.kp_filter_batch(engine.h, b.h, mask), "filter")
    score = (C.c_int64 * (nB * nC))()
    engine._check(L.kp_score_batch(engine.h, b.h, score), "score")
    OL = O.lib()
    idx = (C.c_uint32 * nC)(*range(nC))
    est = (C.c_int32 * nC)()
    bad = []
    for i in range(nB):
        bp = C.pointer(u.bindings[i])
        engine._check(L.kp_max_available_replicas(engine.h, b.h, i, idx, nC, est), "estimate")
        for c in range(nC):
            cp = C.pointer(u.clusters[c])
            fit = OL.kpo_filter(cp, bp, C.byref(opts)) == 0 and not u.clusters[c].deleting
            got = bool((mask[i * W + (c >> 6)] >> (c & 63)) & 1)
            if got != fit:
                bad.append(("filter", i, c, got, fit))
            s = OL.kpo_score(cp, bp, C.byref(opts))
            if score[i * nC + c] != s:
                bad.append(("score", i, c, score[i * nC + c], s))
            e = OL.kpo_max_available_replicas(cp, bp, C.byref(opts), O.FAST)
            if est[c] != e:
                bad.append(("estimate", i, c, est[c], e))
    b.close()
    snap.close()
    assert not bad, f"{len(bad)} mismatches, first: {bad[:8]}"


def test_shard_ranges_match_whole(engine):
    """Scheduling binding ranges separately equals scheduling the whole batch (sharding invariant)."""
    u = synth.Universe(6, 13, 150, 0, 1200)
    opts = api.options()
    whole = gpu_schedule(engine, u, opts)
    parts = []
    for lo, hi in [(0, 1), (1, 500), (500, 1200)]:
        parts += gpu_schedule(engine, u, opts, lo, hi)
    assert whole == parts


def test_repeat_is_deterministic(engine):
    from karmada_amd.engine import Batch, Snapshot
    u = synth.Universe(3, 14, 400, 0, 800)
    snap = Snapshot.from_structs(engine, u.clusters, u.n_clusters, u.names, api.options())
    b = Batch(snap, structs=u.binding_slice(0, u.n_bindings))
    r1 = b.schedule()
    r2 = b.schedule()
    assert r1 == r2
    b.close()
    snap.close()


def test_empty_batch(engine):
    from karmada_amd.engine import Batch, Snapshot
    u = synth.Universe(2, 15, 50, 0, 0)
    snap = Snapshot.from_structs(engine, u.clusters, u.n_clusters, u.names, api.options())
    b = Batch(snap, structs=(u.bindings, 0))
    assert b.schedule() == []


def test_snapshot_update_matches_fresh(engine):
    """kp_snapshot_update on the device: re-packed rows and the refreshed HBM copy
    schedule like a snapshot created from the updated cluster list."""
    from karmada_amd.engine import Batch, Snapshot
    ua = synth.Universe(6, 61, 300, 0, 1500)
    ub = synth.Universe(6, 62, 300, 0, 0)
    opts = api.options()
    idx = sorted(range(0, 300, 7))
    sub_arr = (api.kp_cluster * len(idx))(*[ub.clusters[i] for i in idx])
    mix = (api.kp_cluster * 300)(*[ub.clusters[i] if i in idx else ua.clusters[i] for i in range(300)])
    snap = Snapshot.from_structs(engine, ua.clusters, ua.n_clusters, ua.names, opts)
    snap.update_structs(sub_arr, len(idx))
    got = Batch(snap, structs=ua.binding_slice(0, ua.n_bindings)).schedule()
    ba, n = ua.binding_slice(0, ua.n_bindings)
    compare(got, O.schedule_c(mix, 300, ba, n, opts, O.FAST, 8), "snapshot update")
    snap.close()
