"""FitError diagnosis at the boundary: kp_filter_reasons (the Result of
RunFilterPlugins per pair, runtime/framework.go:93-105) against the oracle's
RunFilterPluginsReason, and FitError.Error() (framework/types.go:67-91) against
the reference's TestFitError_Error (framework/types_test.go:100-160)."""
import ctypes as C
import os

import pytest

from karmada_amd import api, synth
from karmada_amd.engine import Batch, Engine, PKG, Snapshot
import oracle_lib as O

OL = O.lib()
OL.kpo_filter_reason.restype = C.c_uint32


def engine_reasons(engine, u, opts, n_bindings):
    snap = Snapshot.from_structs(engine, u.clusters, u.n_clusters, u.names, opts)
    b = Batch(snap, structs=u.binding_slice(0, n_bindings))
    out = (C.c_uint32 * (n_bindings * u.n_clusters))()
    engine._check(engine.L.kp_filter_reasons(engine.h, b.h, out), "kp_filter_reasons")
    b.close()
    snap.close()
    return out


def oracle_reasons(u, opts, n_bindings):
    return [OL.kpo_filter_reason(C.byref(u.clusters[c]), C.byref(u.bindings[i]), C.byref(opts))
            for i in range(n_bindings) for c in range(u.n_clusters)]


def check(engine, config, seed, nc, nb, opts):
    u = synth.Universe(config, seed, nc, 0, nb)
    got = engine_reasons(engine, u, opts, nb)
    want = oracle_reasons(u, opts, nb)
    bad = [(k // nc, k % nc, got[k], w) for k, w in enumerate(want) if got[k] != w]
    assert not bad, f"{len(bad)} pairs differ, first {bad[:6]}"
    return want


@pytest.mark.parametrize("config,seed,nc,nb", [(6, 31, 120, 150), (4, 4, 200, 60), (3, 3, 150, 60)])
def test_reasons_cpusim(cpusim_engine, config, seed, nc, nb):
    want = check(cpusim_engine, config, seed, nc, nb, api.options())
    if config == 6:  # the edge workload reaches every reason
        kinds = {w & 0xFF for w in want}
        assert {0, 1, 2, 3, 255} <= kinds, kinds


@pytest.mark.parametrize("plugins", [api.PLUGIN_ALL & ~api.PLUGIN_TAINT_TOLERATION, api.PLUGIN_SPREAD_CONSTRAINT, 0])
def test_reasons_cpusim_plugin_sets(cpusim_engine, plugins):
    check(cpusim_engine, 6, 32, 90, 120, api.options(plugins=plugins))


def test_fit_error_message_reference_cases():
    """framework/types_test.go:100-160."""
    assert api.fit_error_message(0, {}) == "0/0 clusters are available: no cluster exists."
    got = api.fit_error_message(3, {"cluster1": ["insufficient CPU", "insufficient memory"],
                                    "cluster2": ["insufficient CPU"], "cluster3": ["taint mismatch"]})
    assert got.startswith("0/3 clusters are available:")
    for r in ("2 insufficient CPU", "1 insufficient memory", "1 taint mismatch"):
        assert r in got
    assert len(got[len("0/3 clusters are available:"):].split(",")) == 3


def test_fit_error_from_engine(cpusim_engine):
    """A binding no cluster fits: the FitError text rebuilt from kp_filter_reasons."""
    from karmada_amd.engine import GenericScheduler
    clusters = [
        {"name": "m1", "taints": [{"key": "a", "value": "x", "effect": "NoSchedule"}],
         "apiEnablements": [{"groupVersion": "apps/v1", "resources": [{"kind": "Deployment"}]}]},
        {"name": "m2", "taints": [{"key": "b", "value": "", "effect": "PreferNoSchedule"},
                                  {"key": "c", "value": "", "effect": "NoExecute"}],
         "apiEnablements": [{"groupVersion": "apps/v1", "resources": [{"kind": "Deployment"}]}]},
        {"name": "m3", "apiEnablements": []},
        {"name": "m4", "deleting": True,
         "apiEnablements": [{"groupVersion": "apps/v1", "resources": [{"kind": "Deployment"}]}]},
        {"name": "m5", "labels": {"env": "dev"},
         "apiEnablements": [{"groupVersion": "apps/v1", "resources": [{"kind": "Deployment"}]}]},
    ]
    binding = {"apiVersion": "apps/v1", "kind": "Deployment", "name": "web", "namespace": "default", "replicas": 2,
               "placement": {"clusterAffinity": {"labelSelector": {"matchLabels": {"env": "prod"}}},
                             "clusterTolerations": [{"key": "z", "operator": "Exists", "effect": "NoSchedule"}]}}
    g = GenericScheduler(cpusim_engine, clusters)
    r = g.schedule([binding])[0]
    assert r.status == api.STATUS_FIT_ERROR and r.arg == 5
    msg = g.fit_error(binding, clusters)
    assert msg == ("0/5 clusters are available: 1 cluster(s) did not have the API resource, "
                   "1 cluster(s) did not match the placement cluster affinity constraint, "
                   "1 cluster(s) had untolerated taint {a=x:NoSchedule}, 1 cluster(s) had untolerated taint {c:NoExecute}.")


@pytest.mark.gpu
def test_reasons_gpu(gpu_engine):
    """Reason histograms of the FIT_ERROR bindings and every pair, GPU vs oracle."""
    want = check(gpu_engine, 6, 31, 700, 300, api.options())
    check(gpu_engine, 4, 4, 5000, 20, api.options())
    assert len(want) == 700 * 300


def test_reasons_cpusim_chunked(cpusim_engine, monkeypatch):
    """The binding chunks of kp_filter_reasons (one reused device buffer) give the
    same words as one pass: chunks of 3 bindings over 50 bindings x 37 clusters."""
    u = synth.Universe(6, 71, 37, 0, 50)
    opts = api.options()
    want = oracle_reasons(u, opts, 50)
    monkeypatch.setenv("KP_REASONS_CHUNK", str(3 * 37))
    got = engine_reasons(cpusim_engine, u, opts, 50)
    assert list(got) == want

