"""kp_snapshot_update: cluster events applied to a packed
snapshot in place give the same placements as a snapshot created from the
updated cluster list (the reference re-snapshots every cluster per Schedule,
cache.go:124-139), checked on the host build of the engine and the oracle."""
import ctypes as C
import os

import pytest

from karmada_amd import api, synth
from karmada_amd.engine import PKG, Batch, Engine, Snapshot
import oracle_lib as O


@pytest.fixture(scope="module")
def engine():
    e = Engine(0, lib_path=os.path.join(PKG, "libkp_cpusim.so"))
    yield e
    e.close()


def mixed(ua, ub, idx):
    """ua's clusters with the indices in idx replaced by ub's (same names, other contents)."""
    arr = (api.kp_cluster * ua.n_clusters)()
    for i in range(ua.n_clusters):
        arr[i] = ub.clusters[i] if i in idx else ua.clusters[i]
    return arr


def subset(ub, idx):
    arr = (api.kp_cluster * len(idx))()
    for k, i in enumerate(sorted(idx)):
        arr[k] = ub.clusters[i]
    return arr


@pytest.mark.parametrize("config,seed_a,seed_b,n_clusters,frac", [
    (6, 41, 42, 200, 0.05), (6, 43, 44, 64, 0.5), (3, 45, 46, 300, 0.1), (4, 47, 48, 400, 0.02), (7, 49, 50, 150, 0.3),
])
def test_update_matches_fresh_snapshot(engine, config, seed_a, seed_b, n_clusters, frac):
    ua = synth.Universe(config, seed_a, n_clusters, 0, 600)
    ub = synth.Universe(config, seed_b, n_clusters, 0, 0)
    opts = api.options()
    idx = set(range(0, n_clusters, max(1, int(1 / frac))))
    snap = Snapshot.from_structs(engine, ua.clusters, ua.n_clusters, ua.names, opts)
    before = Batch(snap, structs=ua.binding_slice(0, ua.n_bindings)).schedule()
    snap.update_structs(subset(ub, idx), len(idx))
    got = Batch(snap, structs=ua.binding_slice(0, ua.n_bindings)).schedule()
    mix = mixed(ua, ub, idx)
    fresh = Snapshot.from_structs(engine, mix, ua.n_clusters, ua.names, opts)
    want = Batch(fresh, structs=ua.binding_slice(0, ua.n_bindings)).schedule()
    assert got == want
    ba, n = ua.binding_slice(0, ua.n_bindings)
    assert want == O.schedule_c(mix, ua.n_clusters, ba, n, opts, O.FAST, 4)
    assert got != before  # the update changed placements
    fresh.close()
    snap.close()


def test_update_rejects_unknown_and_duplicate_names(engine):
    ua = synth.Universe(6, 51, 40, 0, 0)
    ub = synth.Universe(6, 52, 60, 0, 0)  # member-00040.. are not in ua
    snap = Snapshot.from_structs(engine, ua.clusters, ua.n_clusters, ua.names, api.options())
    with pytest.raises(Exception):
        snap.update_structs(subset(ub, {45}), 1)
    two = (api.kp_cluster * 2)(ub.clusters[3], ub.clusters[3])
    with pytest.raises(Exception):
        snap.update_structs(two, 2)
    snap.update_structs(subset(ub, {3, 7}), 2)  # still usable after the rejected calls
    snap.close()


@pytest.mark.parametrize("config,seed_a,seed_b,n_clusters", [(6, 71, 72, 120), (3, 73, 74, 200), (4, 75, 76, 150)])
def test_import_update_matches_fresh(engine, config, seed_a, seed_b, n_clusters):
    """The broadcast path: an imported snapshot (kp_snapshot_import, every non-source
    rank) takes kp_snapshot_update like the snapshot it was exported from."""
    ua = synth.Universe(config, seed_a, n_clusters, 0, 500)
    ub = synth.Universe(config, seed_b, n_clusters, 0, 0)
    opts = api.options()
    idx = set(range(1, n_clusters, 5))
    src = Snapshot.from_structs(engine, ua.clusters, ua.n_clusters, ua.names, opts)
    imp = Snapshot.from_bytes(engine, src.to_bytes(), ua.names)
    imp.update_structs(subset(ub, idx), len(idx))
    got = Batch(imp, structs=ua.binding_slice(0, ua.n_bindings)).schedule()
    mix = mixed(ua, ub, idx)
    fresh = Snapshot.from_structs(engine, mix, ua.n_clusters, ua.names, opts)
    assert got == Batch(fresh, structs=ua.binding_slice(0, ua.n_bindings)).schedule()
    src.update_structs(subset(ub, idx), len(idx))
    assert imp.to_bytes() == src.to_bytes()
    for s in (src, imp, fresh):
        s.close()


def test_import_rejects_corrupt_images(engine):
    """kp_snapshot_import validates every column and offset array: truncated or
    tampered images fail with KP_EINVAL instead of reaching a kernel."""
    import random
    u = synth.Universe(6, 77, 70, 0, 0)
    data = Snapshot.from_structs(engine, u.clusters, u.n_clusters, u.names, api.options()).to_bytes()
    for cut in (8, 100, len(data) // 3, len(data) - 1):
        with pytest.raises(Exception):
            Snapshot.from_bytes(engine, data[:cut], u.names)
    with pytest.raises(Exception):
        Snapshot.from_bytes(engine, data + b"\0", u.names)
    rng = random.Random(5)
    rejected = 0
    for _ in range(300):
        b = bytearray(data)
        i = rng.randrange(8, len(b))
        b[i] ^= 1 << rng.randrange(8)
        try:
            s = Snapshot.from_bytes(engine, bytes(b), u.names)
            s.close()  # a flip inside a value column can be a valid image
        except Exception:
            rejected += 1
    assert rejected > 0


def test_region_set_change_is_reported(engine):
    """A region-spread batch packed before an update that changes the region set
    is refused (KP_ESTATE) instead of writing past its region buffers."""
    from karmada_amd.engine import EngineError
    ua = synth.Universe(4, 78, 120, 0, 200)
    snap = Snapshot.from_structs(engine, ua.clusters, ua.n_clusters, ua.names, api.options())
    b = Batch(snap, structs=ua.binding_slice(0, ua.n_bindings))
    w = api.World()
    c = w.cluster({"name": ua.names[3], "region": "region-zz-new",
                   "resourceSummary": {"allocatable": {"cpu": "10", "pods": "100"}}})
    arr = (api.kp_cluster * 1)(c)
    assert snap.update_structs(arr, 1) is True
    with pytest.raises(EngineError):
        b.schedule()
    b2 = Batch(snap, structs=ua.binding_slice(0, ua.n_bindings))
    assert len(b2.schedule()) == ua.n_bindings
    snap.close()
