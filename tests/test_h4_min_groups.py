"""SURVEY hazard H4 through the whole engine: calcGroupScore's
int64(math.Ceil(float64(Replicas) / float64(MinGroups))) with a region constraint
whose MinGroups is 0 (group_clusters.go:247-249): +Inf (NaN at Replicas 0) converts
to MinInt64 on amd64, so target*1000 wraps and the walk's "sum >= target" holds at
the first cluster. Synthetic config 11 (config-4 clusters, region and cluster
constraints with MinGroups 0, Divided and Duplicated bindings, 20% with spec.Clusters)
runs through kp_schedule_batch against the oracle, which counts the conversions
that took that branch (kpo_h4_hits), so the test also shows the path ran.
Parity only: no reference test pins the amd64 conversion."""
import pytest

from karmada_amd import api, synth
import oracle_lib as O


def check(engine, seed, n_clusters, n_bindings):
    from karmada_amd.engine import Batch, Snapshot
    u = synth.Universe(11, seed, n_clusters, 0, n_bindings)
    opts = api.options()
    L = O.lib()
    L.kpo_h4_hits(1)
    want = O.schedule_c(u.clusters, u.n_clusters, u.bindings, u.n_bindings, opts, O.FAST, 1)
    hits = L.kpo_h4_hits(1)
    snap = Snapshot.from_structs(engine, u.clusters, u.n_clusters, u.names, opts)
    b = Batch(snap, structs=u.binding_slice(0, u.n_bindings))
    got = b.schedule()
    t = engine.stage_times()
    b.close()
    snap.close()
    bad = [i for i in range(len(want)) if got[i] != want[i]]
    assert not bad, f"{len(bad)}/{len(want)} differ; first {bad[0]}: got={got[bad[0]]} want={want[bad[0]]}"
    ok = sum(1 for r in want if r["status"] == 0)
    return hits, ok, t


def test_h4_host_build(cpusim_engine):
    hits, ok, t = check(cpusim_engine, 111, 400, 1500)
    assert hits > 100 and ok > 500, (hits, ok)
    assert t["n_region"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n_clusters,n_bindings", [(111, 400, 3000), (112, 5000, 3000)])
def test_h4_gpu(gpu_engine, seed, n_clusters, n_bindings):
    hits, ok, t = check(gpu_engine, seed, n_clusters, n_bindings)
    assert hits > 200 and ok > 1000, (hits, ok)
    assert t["n_region"] > 0 and t["n_cluster"] > 0
