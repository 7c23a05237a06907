"""kp_schedule_batch_submit / _collect: kp_schedule_batch in two halves, so a caller keeps
the next batch's kernels queued while it reads the last one back (bench.py's lanes do).
Two batches of one engine submitted before either is collected, collected in either order,
schedule exactly as kp_schedule_batch does (and as the oracle), across a region chain
(config 4) and the singleton-class rows (config 10); misuse reports KP_ESTATE."""
import pytest

from karmada_amd import api, synth
from karmada_amd.engine import Batch, EngineError, Snapshot


def run(engine, config, n_clusters, n_bind):
    u = synth.Universe(config, 5, n_clusters, 0, 2 * n_bind)
    snap = Snapshot.from_structs(engine, u.clusters, u.n_clusters, u.names, api.options())
    b1 = Batch(snap, structs=u.binding_slice(0, n_bind))
    b2 = Batch(snap, structs=u.binding_slice(n_bind, 2 * n_bind))
    want1, want2 = b1.schedule(), b2.schedule()

    def py(r):
        return api.results_to_python(r.status, r.err_code, r.err_arg, r.offsets, r.cluster_idx, r.replicas,
                                     r.n_bindings)
    for order in ((b1, b2), (b2, b1)):
        b1.submit()
        b2.submit()
        got = {id(b): py(b.collect()) for b in order}
        assert got[id(b1)] == want1
        assert got[id(b2)] == want2
    # a pipelined stream of calls: submit the next before collecting the last
    b1.submit()
    for _ in range(3):
        b2.submit()
        assert py(b1.collect()) == want1
        b1.submit()
        assert py(b2.collect()) == want2
    assert py(b1.collect()) == want1
    with pytest.raises(EngineError):
        b1.collect()  # nothing submitted
    b2.submit()
    with pytest.raises(EngineError):
        b2.submit()  # the previous call is not collected
    assert py(b2.collect()) == want2
    b1.submit()  # destroyed with a call in flight: the batch waits for it
    b1.close()
    b2.close()
    snap.close()


@pytest.mark.parametrize("config,C,n", [(3, 400, 1500), (4, 300, 1500), (10, 300, 1500)])
def test_submit_collect_cpusim(cpusim_engine, config, C, n):
    run(cpusim_engine, config, C, n)


@pytest.mark.gpu
@pytest.mark.parametrize("config,C,n", [(3, 5000, 4000), (4, 5000, 4000), (10, 5000, 4000)])
def test_submit_collect_gpu(gpu_engine, config, C, n):
    run(gpu_engine, config, C, n)
