"""kp_pack_cache: packed binding records reused across scheduling cycles (VERDICT r5
item 6). The reference re-runs Schedule for bindings whose spec did not change
(pkg/scheduler/scheduler.go:437-468: Duplicated / non-workload bindings on every
reconcile, terminating target clusters, requeued failures); a spec change moves
metadata.generation. A batch created through kp_batch_create_keyed must be the batch
kp_batch_create packs from the same bindings (kp_batch_digest over headers, pools,
routes and estimator classes) and schedule identically, whichever records it reused;
a changed generation or scheduler status field, or a snapshot whose dictionaries grew,
re-packs."""
import ctypes as C
import os
import random

import pytest

from karmada_amd import api, synth
from karmada_amd.engine import Batch, PackCache, Snapshot


def copy_bindings(src, idx):
    arr = (api.kp_binding * max(1, len(idx)))()
    for j, i in enumerate(idx):
        arr[j] = src[i]
    return arr


def run_case(engine, n_bind=9000, n_clusters=300, schedule_check=True):
    os.environ["KP_PACK_THREADS"] = "3"
    try:
        u = synth.Universe(6, 11, n_clusters, 0, n_bind)
        opts = api.options()
        snap = Snapshot.from_structs(engine, u.clusters, u.n_clusters, u.names, opts)
        n = u.n_bindings
        gens = [1 + (i % 7) for i in range(n)]
        keys = api.binding_keys(u.bindings, n, gens)
        fresh = Batch(snap, structs=(u.bindings, n))
        d0 = fresh.digest()
        cache = PackCache(engine)
        cold = Batch(snap, structs=(u.bindings, n), cache=cache, keys=keys)
        assert cold.digest() == d0
        st = cache.stats()
        assert st["last_hits"] == 0 and st["entries"] == n, st
        warm = Batch(snap, structs=(u.bindings, n), cache=cache, keys=keys)
        assert warm.digest() == d0
        assert cache.stats()["last_hits"] == n
        if schedule_check:
            assert warm.schedule() == fresh.schedule()
        for b in (fresh, cold, warm):
            b.close()

        # the next cycle: shuffled, some bindings with a new generation, some with a
        # changed status (lastScheduledTime, observed affinity name), some new ones
        rng = random.Random(5)
        idx = list(range(n))
        rng.shuffle(idx)
        idx = idx[: n - 500]
        arr = copy_bindings(u.bindings, idx)
        g2 = [gens[i] for i in idx]
        bumped = set(rng.sample(range(len(idx)), 700))
        for j in bumped:
            g2[j] += 1
        touched = set(rng.sample(range(len(idx)), 300)) - bumped
        for j in touched:
            arr[j].has_last_scheduled_time = 1
            arr[j].last_scheduled_time_ns = arr[j].last_scheduled_time_ns + 12345
        names = set(rng.sample(range(len(idx)), 100)) - bumped - touched
        keep = []
        for j in names:
            nm = C.create_string_buffer(b"other-term")
            keep.append(nm)
            arr[j].observed_affinity_name = api.kp_str(C.cast(nm, C.c_char_p), 10)
        k2 = api.binding_keys(arr, len(idx), g2)
        want = Batch(snap, structs=(arr, len(idx)))
        got = Batch(snap, structs=(arr, len(idx)), cache=cache, keys=k2)
        assert got.digest() == want.digest()
        assert cache.stats()["last_hits"] == len(idx) - len(bumped) - len(touched) - len(names)
        if schedule_check:
            assert got.schedule() == want.schedule()
        got.close()
        want.close()

        # a snapshot whose dictionaries grew: the records resolved against the old ones
        assert snap.update([{"name": u.names[0], "labels": {"brand-new-key": "v"},
                             "resourceSummary": {"allocatable": {"cpu": "8", "pods": "110"}}}])  # dict_grew
        after = Batch(snap, structs=(u.bindings, n), cache=cache, keys=keys)
        assert cache.stats()["last_hits"] == 0
        fresh2 = Batch(snap, structs=(u.bindings, n))
        assert after.digest() == fresh2.digest()
        after.close()
        fresh2.close()
        cache.close()
        snap.close()
    finally:
        os.environ.pop("KP_PACK_THREADS", None)


def test_pack_cache_reuse_matches_fresh_pack(cpusim_engine):
    run_case(cpusim_engine)


def test_pack_cache_keys_required(cpusim_engine):
    u = synth.Universe(3, 3, 64, 0, 16)
    snap = Snapshot.from_structs(cpusim_engine, u.clusters, u.n_clusters, u.names, api.options())
    h = C.c_void_p()
    L = cpusim_engine.L
    assert L.kp_batch_create_keyed(cpusim_engine.h, snap.h, u.bindings, None, u.n_bindings, None, C.byref(h)) != 0
    snap.close()


@pytest.mark.gpu
def test_pack_cache_reuse_matches_fresh_pack_gpu(gpu_engine):
    run_case(gpu_engine, n_bind=9000, n_clusters=300)
