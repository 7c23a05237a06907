"""k_select_top phase stamps (diagnostic build libkp_stamps.so, -DKP_STAMPS): config 3,
one batch at a time, both slices on one stream. Prints the per-phase s_memtime sums the
engine dumps to stderr (kp_select.h KP_STAMP ids) for a few steps."""
import os
import sys
import time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ.setdefault("KP_TOP_SPLIT", "0")
from karmada_amd import api, synth  # noqa: E402
from karmada_amd.engine import Batch, Engine, Snapshot  # noqa: E402
cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
lib = sys.argv[2] if len(sys.argv) > 2 else "karmada_amd/libkp_stamps.so"
C_, B = synth.CONFIGS[cfg]
u = synth.Universe(cfg, cfg, C_, 0, B)
e = Engine(0, lib_path=os.path.join(ROOT, lib))
snap = Snapshot.from_structs(e, u.clusters, u.n_clusters, u.names, api.options())
b = Batch(snap, structs=u.binding_slice(0, B))
for i in range(4):
    t = time.perf_counter()
    b.schedule_raw()
    dt = (time.perf_counter() - t) * 1e3
    st = e.stage_times()
    print(round(dt, 3), "top", round(st["top_kernel_ms"], 3), flush=True)
