"""Binding packing + upload timing on the GPU box (KP_PACK_TIMING breakdown)."""
import os
import resource
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ.setdefault("KP_PACK_TIMING", "1")
from karmada_amd import api, synth  # noqa: E402
from karmada_amd.engine import Batch, Engine, Snapshot  # noqa: E402

eng = Engine(0, lib_path=os.environ["KP_LIB"]) if os.environ.get("KP_LIB") else Engine(0)
u = synth.Universe(3, 3, 5000, 0, 100000)
snap = Snapshot.from_structs(eng, u.clusters, u.n_clusters, u.names, api.options())
structs = u.binding_slice(0, u.n_bindings)
for i in range(5):
    r0 = resource.getrusage(resource.RUSAGE_SELF)
    t = time.perf_counter()
    b = Batch(snap, structs=structs)
    t1 = time.perf_counter()
    b.schedule_raw()
    t2 = time.perf_counter()
    b.close()
    t3 = time.perf_counter()
    r1 = resource.getrusage(resource.RUSAGE_SELF)
    print("create %.1f ms schedule %.1f ms close %.1f ms | cpu user %.0f ms sys %.0f ms" %
          ((t1 - t) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, (r1.ru_utime - r0.ru_utime) * 1e3,
           (r1.ru_stime - r0.ru_stime) * 1e3), flush=True)
print("cpus", os.cpu_count(), len(os.sched_getaffinity(0)))
