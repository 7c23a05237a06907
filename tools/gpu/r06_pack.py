"""Host-side batch creation on the GPU box: fresh packing against kp_pack_cache reuse
(config 3, 100k bindings), with the engine's pack timing (KP_PACK_TIMING)."""
import os
import sys
import time
import numpy as np
os.environ.setdefault("KP_PACK_TIMING", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import ctypes as C  # noqa: E402
from karmada_amd import api, synth  # noqa: E402
from karmada_amd.engine import Batch, Engine, PackCache, Snapshot  # noqa: E402
u = synth.Universe(3, 3, 5000, 0, 100000)
e = Engine(0)
snap = Snapshot.from_structs(e, u.clusters, u.n_clusters, u.names, api.options())
n = u.n_bindings
st = (u.bindings, n)
for i in range(3):
    t = time.perf_counter()
    Batch(snap, structs=st).close()
    print("fresh", round(1e3 * (time.perf_counter() - t), 2), "ms", flush=True)
keys = api.binding_keys(u.bindings, n, [1] * n)
c = PackCache(e)
for i in range(4):
    t = time.perf_counter()
    Batch(snap, structs=st, cache=c, keys=keys).close()
    print("keyed all-same", round(1e3 * (time.perf_counter() - t), 2), "ms", c.stats(), flush=True)
kdt = np.dtype({"names": ["gen"], "formats": ["<i8"], "offsets": [16], "itemsize": C.sizeof(api.kp_binding_key)})
for cyc in range(1, 4):
    ks = (api.kp_binding_key * n).from_buffer_copy(keys)
    g = np.frombuffer(ks, dtype=kdt)["gen"]
    g[(np.arange(n) * 2654435761 + cyc * 40503) % 1000 < 100] += cyc
    t = time.perf_counter()
    Batch(snap, structs=st, cache=c, keys=ks).close()
    print("keyed churn 10%", round(1e3 * (time.perf_counter() - t), 2), "ms", c.stats(), flush=True)
