"""Reference filter/score plugin tests (tests/golden/plugins.json, transcribed from
pkg/scheduler/framework/plugins/*/*_test.go and pkg/apis/cluster/v1alpha1/
cluster_helper_test.go) through the oracle, the engine's host build
(libkp_cpusim.so) and, under -m gpu, libkp.so on the MI355X.

Each case enables only the plugin under test (the --plugins flag,
cmd/scheduler/app/options/options.go:163), so the engine's fused filter answers
exactly that plugin's Filter/Score.
"""
import ctypes as C
import json
import os

import pytest

import oracle_lib as O
from karmada_amd import api

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
PLUG = json.load(open(os.path.join(GOLDEN, "plugins.json")))
BIT = {"APIEnablement": api.PLUGIN_API_ENABLEMENT, "TaintToleration": api.PLUGIN_TAINT_TOLERATION,
       "ClusterAffinity": api.PLUGIN_CLUSTER_AFFINITY, "SpreadConstraint": api.PLUGIN_SPREAD_CONSTRAINT,
       "ClusterLocality": api.PLUGIN_CLUSTER_LOCALITY, "ClusterEviction": api.PLUGIN_CLUSTER_EVICTION}


def ids(cases):
    return ["%s: %s" % (c["plugin"], c["name"]) for c in cases]


def oracle_filter(case):
    w = api.World()
    c = w.cluster(case["cluster"])
    b = w.binding(case["binding"])
    o = api.options(plugins=BIT[case["plugin"]])
    return O.lib().kpo_filter(C.byref(c), C.byref(b), C.byref(o)) == 0


def oracle_score(case):
    w = api.World()
    c = w.cluster(case["cluster"])
    b = w.binding(case["binding"])
    o = api.options(plugins=BIT[case["plugin"]])
    return O.lib().kpo_score(C.byref(c), C.byref(b), C.byref(o))


def engine_filter(engine, case):
    from karmada_amd.engine import GenericScheduler
    g = GenericScheduler(engine, [case["cluster"]], api.options(plugins=BIT[case["plugin"]]))
    return g.filter([case["binding"]])[0] == [case["cluster"]["name"]]


def engine_score(engine, case):
    from karmada_amd.engine import GenericScheduler
    g = GenericScheduler(engine, [case["cluster"]], api.options(plugins=BIT[case["plugin"]]))
    return g.score([case["binding"]])[0][0]


@pytest.mark.parametrize("case", PLUG["filters"], ids=ids(PLUG["filters"]))
def test_filter_oracle(case):
    assert oracle_filter(case) == case["fit"]


@pytest.mark.parametrize("case", PLUG["scores"], ids=ids(PLUG["scores"]))
def test_score_oracle(case):
    assert oracle_score(case) == case["score"]


@pytest.mark.parametrize("case", PLUG["filters"], ids=ids(PLUG["filters"]))
def test_filter_cpusim(cpusim_engine, case):
    assert engine_filter(cpusim_engine, case) == case["fit"]


@pytest.mark.parametrize("case", PLUG["scores"], ids=ids(PLUG["scores"]))
def test_score_cpusim(cpusim_engine, case):
    assert engine_score(cpusim_engine, case) == case["score"]


@pytest.mark.gpu
def test_filter_score_gpu(gpu_engine):
    bad = [c["name"] for c in PLUG["filters"] if engine_filter(gpu_engine, c) != c["fit"]]
    bad += [c["name"] for c in PLUG["scores"] if engine_score(gpu_engine, c) != c["score"]]
    assert not bad, bad


# Test_extractClusterFields (pkg/util/selector_test.go:927-986): the field set a
# cluster exposes to FieldSelector requirements (selector.go:187-199) is {provider,
# region} for the non-empty ones. extractClusterFields is internal, so each table
# row is observed through ClusterAffinity field selectors: Exists on a field
# passes exactly when the row's want set holds it, and In [value] on each held
# field passes.
EXTRACT_FIELDS = [
    ("empty", {}, {}),
    ("provider is set", {"provider": "foo"}, {"provider": "foo"}),
    ("region is set", {"region": "foo"}, {"region": "foo"}),
    ("all are set", {"provider": "foo", "region": "bar"}, {"provider": "foo", "region": "bar"}),
]


def field_cases():
    out = []
    for name, spec, want in EXTRACT_FIELDS:
        cluster = {"name": "member1", "labels": {}, **spec}
        probes = [([{"key": f, "operator": "Exists", "values": []}], f in want) for f in ("provider", "region")]
        probes += [([{"key": f, "operator": "In", "values": [v]}], True) for f, v in want.items()]
        probes += [([{"key": f, "operator": "DoesNotExist", "values": []}], f not in want) for f in ("provider", "region")]
        for exprs, fit in probes:
            binding = {"placement": {"clusterAffinity": {"fieldSelector": {"matchExpressions": exprs}}}}
            out.append({"name": f"{name}: {exprs[0]['key']} {exprs[0]['operator']}", "plugin": "ClusterAffinity",
                        "binding": binding, "cluster": cluster, "fit": fit})
    return out


FIELD_CASES = field_cases()


@pytest.mark.parametrize("case", FIELD_CASES, ids=[c["name"] for c in FIELD_CASES])
def test_extract_cluster_fields(cpusim_engine, case):
    assert oracle_filter(case) == case["fit"]
    assert engine_filter(cpusim_engine, case) == case["fit"]


@pytest.mark.gpu
def test_extract_cluster_fields_gpu(gpu_engine):
    bad = [c["name"] for c in FIELD_CASES if engine_filter(gpu_engine, c) != c["fit"]]
    assert not bad, bad
