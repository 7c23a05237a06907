"""CPU parity of the engine's own code: libkp_cpusim.so runs engine.cpp and the
kernel bodies of kp_kernels.h (1-thread block policy) on the host, checked
against the oracle. The GPU build of the same bodies is checked in
tests/test_gpu_parity.py; this file keeps the logic covered on every CPU run."""
import os

import pytest

from karmada_amd import api, synth
from karmada_amd.engine import Batch, Engine, Snapshot, PKG
import oracle_lib as O

CPUSIM = os.path.join(PKG, "libkp_cpusim.so")


@pytest.fixture(scope="module")
def engine():
    os.environ.setdefault("KP_CPUSIM_THREADS", "8")
    e = Engine(0, lib_path=CPUSIM)
    yield e
    e.close()


def run(engine, u, opts, lo=0, hi=None, rows=False, times=None):
    """Schedules bindings [lo, hi); rows=True forces the per-binding pair rows
    (KP_PAIR_ROWS=1) instead of the bitset filter + estimator classes, times (a
    list) receives the call's kp_stage_times."""
    hi = u.n_bindings if hi is None else hi
    snap = Snapshot.from_structs(engine, u.clusters, u.n_clusters, u.names, opts)
    b = Batch(snap, structs=u.binding_slice(lo, hi))
    if rows:
        os.environ["KP_PAIR_ROWS"] = "1"
    try:
        out = b.schedule()
    finally:
        os.environ.pop("KP_PAIR_ROWS", None)
    if times is not None:
        times.append(engine.stage_times())
    b.close()
    snap.close()
    return out


def compare(got, want, label):
    bad = [i for i, (g, w) in enumerate(zip(got, want)) if g != w]
    assert len(got) == len(want)
    if bad:
        msg = [f"{label}: {len(bad)}/{len(want)} differ"]
        for i in bad[:4]:
            msg += [f"  {i}: sim={got[i]}", f"  {i}: ref={want[i]}"]
        pytest.fail("\n".join(msg))


@pytest.mark.parametrize("rows", [False, True], ids=["bits", "rows"])
@pytest.mark.parametrize("config,seed,n_clusters,n_bindings", [
    (1, 1, 10, 1000), (2, 2, 300, 400), (3, 3, 200, 300), (4, 4, 400, 500),
    (6, 6, 120, 1500), (6, 7, 40, 1500), (6, 8, 1, 200), (6, 9, 257, 600),
    (7, 17, 300, 400), (7, 18, 13, 300), (5, 5, 500, 600),
    (8, 4, 64, 300), (8, 7, 24, 200),
])
def test_cpusim_schedule_parity(engine, config, seed, n_clusters, n_bindings, rows):
    u = synth.Universe(config, seed, n_clusters, 0, n_bindings)
    opts = api.options()
    ba, n = u.binding_slice(0, n_bindings)
    want = O.schedule_c(u.clusters, u.n_clusters, ba, n, opts, O.FAST, 8)
    times = []
    compare(run(engine, u, opts, rows=rows, times=times), want, f"config {config} seed {seed}")
    if config in (2, 3, 5, 7):  # fast estimator instances
        assert times[0]["bits"] == int(not rows)
    if config in (4, 5) and not rows:  # cluster spread without spec.Clusters: the class-order selection
        assert 0 < times[0]["n_cluster_order"] <= times[0]["n_cluster"]
    if config == 4 and not rows:
        assert 0 < times[0]["n_region_order"] <= times[0]["n_region"]


@pytest.mark.parametrize("prop,plugins,gate", [
    (True, api.PLUGIN_ALL, True),
    (False, api.PLUGIN_ALL & ~api.PLUGIN_TAINT_TOLERATION, False),
    (False, 0, True),
])
def test_cpusim_options(engine, prop, plugins, gate):
    u = synth.Universe(6, 21, 90, 0, 800)
    opts = api.options(empty_workload_propagation=prop, models_gate=gate, plugins=plugins)
    ba, n = u.binding_slice(0, u.n_bindings)
    want = O.schedule_c(u.clusters, u.n_clusters, ba, n, opts, O.FAST, 8)
    compare(run(engine, u, opts), want, f"options {prop} {plugins} {gate}")


def test_cpusim_overflow_tiers_large_c(engine):
    """Config 6 at C = 5000: overflow-tier bindings take k_slow's exact serial path with
    candidate lists of ~5k, run by 8 concurrent host 'workgroups'. Guards the serial
    scratch sizing (serial_scratch_bytes once undercounted its u32 arrays, so a slot's
    result list ran into the next workgroup's slot)."""
    u = synth.Universe(6, 13, 5000, 0, 4000)
    opts = api.options()
    ba, n = u.binding_slice(0, 4000)
    want = O.schedule_c(u.clusters, u.n_clusters, ba, n, opts, O.FAST, 8)
    compare(run(engine, u, opts, 0, 4000), want, "config 6 seed 13 C=5000")


def test_cpusim_parallel_packing(engine):
    """kp_batch_create packs on several host threads (one per 4096 bindings) and
    rebases every pool reference: the results equal a one-thread pack and the oracle."""
    u = synth.Universe(6, 41, 60, 0, 20000)
    opts = api.options()
    os.environ["KP_PACK_THREADS"] = "1"
    try:
        one = run(engine, u, opts)
    finally:
        os.environ.pop("KP_PACK_THREADS", None)
    os.environ["KP_PACK_THREADS"] = "5"
    try:
        many = run(engine, u, opts)
    finally:
        os.environ.pop("KP_PACK_THREADS", None)
    assert many == one
    ba, n = u.binding_slice(0, u.n_bindings)
    compare(many, O.schedule_c(u.clusters, u.n_clusters, ba, n, opts, O.FAST, 8), "parallel packing")


@pytest.mark.parametrize("rows", [False, True], ids=["bits", "rows"])
@pytest.mark.parametrize("config,seed,n_clusters,n_bindings,multi", [
    (9, 1, 300, 600, True), (9, 2, 120, 300, False), (6, 3, 120, 1500, True),
])
def test_cpusim_multi_templates(engine, config, seed, n_clusters, n_bindings, multi, rows):
    """MultiplePodTemplatesScheduling on: MaxAvailableComponentSets class rows
    (k_sets_rows) and SelectBestClusters' one-set need (common.go:42-46)."""
    u = synth.Universe(config, seed, n_clusters, 0, n_bindings)
    opts = api.options(multi_templates=multi)
    ba, n = u.binding_slice(0, n_bindings)
    want = O.schedule_c(u.clusters, u.n_clusters, ba, n, opts, O.FAST, 8)
    compare(run(engine, u, opts, rows=rows), want, f"multi {multi} config {config} seed {seed}")


def test_cpusim_region_host_dfs(engine):
    """selectGroups on the host (KP_REGION_HOST=1: the route of snapshots with more
    regions than the device DFS arrays, and of bindings past its node budget) gives
    the device DFS's results: config 4's region spread against the oracle."""
    u = synth.Universe(4, 44, 400, 0, 400)
    opts = api.options()
    want = O.schedule_c(u.clusters, u.n_clusters, u.bindings, u.n_bindings, opts, O.FAST, 8)
    os.environ["KP_REGION_HOST"] = "1"
    try:
        got = run(engine, u, opts)
    finally:
        os.environ.pop("KP_REGION_HOST", None)
    compare(got, want, "region host DFS")


@pytest.mark.parametrize("top_env", [{"KP_TOP_CAP": "64"}, {"KP_TOP": "0"}, {"KP_TOP_CAP_MID": "64"},
                                     {"KP_TOP_CAP_MID": "64", "KP_TOP_CAP": "128"}],
                         ids=["cap64", "off", "mid64", "mid64-cap128"])
def test_cpusim_top_subsets(top_env):
    """k_select_top (kp_top.h) at its smallest subset capacity (most bindings hand back
    to the full-candidate kernel through the device fallback list), switched off, and
    with the large slice run first at a small capacity (KP_TOP_CAP_MID: the overflow list
    run again at the full capacity, its own overflow to the full-candidate kernel): the
    same placements as the oracle every way."""
    old = {k: os.environ.get(k) for k in top_env}
    os.environ.update(top_env)
    try:
        e = Engine(0, lib_path=CPUSIM)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    try:
        for config, seed, C_, B_ in [(3, 53, 400, 600), (7, 54, 300, 300), (6, 55, 150, 800)]:
            u = synth.Universe(config, seed, C_, 0, B_)
            opts = api.options()
            want = O.schedule_c(u.clusters, u.n_clusters, u.bindings, u.n_bindings, opts, O.FAST, 8)
            times = []
            compare(run(e, u, opts, times=times), want, f"{top_env} config {config}")
            if top_env.get("KP_TOP") == "0":
                assert times[0]["n_top"] == 0
            elif top_env.get("KP_TOP_CAP") == "64":
                assert times[0]["n_top_fallback"] > 0
            else:
                assert times[0]["n_top"] > 0
    finally:
        e.close()


@pytest.mark.parametrize("slow_env", [{"KP_SLOW_ORDER": "1"}, {"KP_SLOW_ORDER": "0"}, {"KP_TOP_WG": "1"}],
                         ids=["order", "sort", "top-wg"])
def test_cpusim_slow_order_and_top_wg(slow_env):
    """k_slow's candidate order from the class orders (kp_kernels.h slow_items_from_order:
    the filtered class order, spec.Clusters merged in) against the bitonic sort it replaces,
    and the workgroup form of k_select_top for the large subsets, on config 7 (Aggregated
    tie groups straddling the cut: every tie binding goes through k_slow, 20% with
    spec.Clusters) and config 3: the oracle's placements every way."""
    old = {k: os.environ.get(k) for k in slow_env}
    os.environ.update(slow_env)
    try:
        e = Engine(0, lib_path=CPUSIM)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    try:
        for config, seed, C_, B_ in [(7, 71, 400, 500), (3, 72, 500, 700)]:
            u = synth.Universe(config, seed, C_, 0, B_)
            opts = api.options()
            want = O.schedule_c(u.clusters, u.n_clusters, u.bindings, u.n_bindings, opts, O.FAST, 8)
            compare(run(e, u, opts), want, f"{slow_env} config {config}")
    finally:
        e.close()


def test_cpusim_sets_overflow_is_per_binding(engine):
    """A component-set simulation that outgrows its node runs (KP_SETS_RUNS_CAP=1 here;
    kSetsRunsMax on the device) fails only the bindings of that component-set class
    (KP_ERR_SETS_CAPACITY, arg = a caller cluster index); every other binding keeps
    the oracle's result (the whole batch used to fail with KP_ENOTSUP)."""
    u = synth.Universe(9, 1, 300, 0, 600)
    opts = api.options(multi_templates=True)
    want = O.schedule_c(u.clusters, u.n_clusters, u.bindings, u.n_bindings, opts, O.FAST, 8)
    os.environ["KP_SETS_RUNS_CAP"] = "1"
    try:
        got = run(engine, u, opts)
    finally:
        os.environ.pop("KP_SETS_RUNS_CAP", None)
    failed = [i for i, g in enumerate(got) if g["err"] == 15]
    assert failed, "no component-set class overflowed: the test needs another cap or universe"
    for i in failed:
        assert got[i]["status"] == api.STATUS_ERROR and got[i]["targets"] == [] and 0 <= got[i]["arg"] < 300
    ok = [i for i in range(len(got)) if i not in set(failed)]
    assert ok  # (most of the multi-template bindings overflow at a cap of one run)
    compare([got[i] for i in ok], [want[i] for i in ok], "sets overflow: the other bindings")


def test_cpusim_kernel_times():
    """kp_engine_set_profile: every kernel of the step is timed by its own event pair and
    reported by name with its launches and the bindings it covered (the bench ranks the
    step's kernels by these times); results are unchanged with profiling on."""
    e = Engine(0, lib_path=CPUSIM)
    try:
        e.set_profile(True)
        for config, seed, C_, B_, must in [
            (3, 3, 200, 300, {"k_est_class_m8", "k_filter", "k_class_order", "k_select_top", "k_offsets", "k_compact"}),
            (4, 4, 400, 500, {"k_spread_order", "k_region_a_order", "k_region_groups"}),
            (8, 4, 64, 300, {"k_slow"}),
        ]:
            u = synth.Universe(config, seed, C_, 0, B_)
            opts = api.options()
            want = O.schedule_c(u.clusters, u.n_clusters, u.bindings, u.n_bindings, opts, O.FAST, 8)
            compare(run(e, u, opts), want, f"profiled config {config}")
            kt = e.kernel_times()
            assert must <= set(kt), (config, sorted(kt))
            assert all(v["launches"] >= 1 and v["ms"] >= 0 for v in kt.values())
            assert kt["k_filter"]["units"] == B_ if "k_filter" in kt else True
            if config == 8:
                assert kt["k_slow"]["units"] == e.stage_times()["n_slow"] > 0
        e.set_profile(False)
        u = synth.Universe(3, 3, 200, 0, 100)
        run(e, u, api.options())
        assert e.kernel_times() == {}
    finally:
        e.close()


@pytest.mark.parametrize("cap", [None, "64", "mid64"], ids=["cap", "cap64", "mid64"])
@pytest.mark.parametrize("config,seed,n_clusters,n_bindings", [
    (3, 3, 1000, 2000), (7, 17, 300, 1500), (6, 9, 700, 2000), (8, 4, 64, 1000), (8, 5, 16, 600), (10, 10, 2000, 1500),
])
def test_cpusim_top_histogram(config, seed, n_clusters, n_bindings, cap):
    """k_select_top without class orders (KP_ORDER_AMORT forces it; config 10 takes it by
    itself: about one estimator class per binding): each binding's feasible votes are
    thresholded by an octave histogram instead of walking an order (kp_top.h), including
    the wrap and negative-vote fallbacks of config 8."""
    u = synth.Universe(config, seed, n_clusters, 0, n_bindings)
    opts = api.options()
    os.environ["KP_ORDER_AMORT"] = "1000000"
    if cap == "mid64":  # (read at engine creation) the large slice first at 64, then at full capacity
        os.environ["KP_TOP_CAP_MID"] = "64"
    elif cap:  # a small subset capacity: the list compactions and overflow
        os.environ["KP_TOP_CAP"] = cap
    times = []
    try:
        e = Engine(0, lib_path=CPUSIM)
        got = run(e, u, opts, times=times)
        e.close()
    finally:
        os.environ.pop("KP_ORDER_AMORT", None)
        os.environ.pop("KP_TOP_CAP", None)
        os.environ.pop("KP_TOP_CAP_MID", None)
    assert times[0]["n_top"] > 0
    want = O.schedule_c(u.clusters, u.n_clusters, u.bindings, u.n_bindings, opts, O.FAST, 8)
    compare(got, want, f"histogram config {config}")
