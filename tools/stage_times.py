import sys, time
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from karmada_amd import api, synth
from karmada_amd.engine import Engine, Batch, Snapshot
u = synth.Universe(3, 3, 5000, 0, 100000)
e = Engine(0)
snap = Snapshot.from_structs(e, u.clusters, u.n_clusters, u.names, api.options())
b = Batch(snap, structs=u.binding_slice(0, 100000))
for i in range(4):
    t = time.perf_counter(); b.schedule_raw(); dt = (time.perf_counter() - t) * 1e3
    print(round(dt, 3), {k: round(v, 3) for k, v in e.stage_times().items() if isinstance(v, float)})
