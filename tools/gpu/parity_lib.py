"""Parity of one engine library against the oracle on seeded universes (a GPU-box
diagnostic for a candidate build kept beside the in-tree one):

    python tools/gpu/parity_lib.py <lib.so> config:seed:clusters:bindings ...
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from karmada_amd import api, synth  # noqa: E402
from karmada_amd.engine import Batch, Engine, Snapshot  # noqa: E402
import oracle_lib as O  # noqa: E402


def main():
    e = Engine(0, lib_path=sys.argv[1])
    bad_total = 0
    for spec in sys.argv[2:]:
        cfg, seed, C_, B_ = (int(x) for x in spec.split(":"))
        u = synth.Universe(cfg, seed, C_, 0, B_)
        opts = api.options()
        snap = Snapshot.from_structs(e, u.clusters, u.n_clusters, u.names, opts)
        b = Batch(snap, structs=u.binding_slice(0, B_))
        got = b.schedule()
        b.close()
        snap.close()
        want = O.schedule_c(u.clusters, u.n_clusters, u.bindings, u.n_bindings, opts, O.FAST, 8)
        bad = [i for i, (g, w) in enumerate(zip(got, want)) if g != w]
        bad_total += len(bad)
        print(f"{spec}: {len(bad)}/{B_} differ {bad[:8]}", flush=True)
    e.close()
    sys.exit(1 if bad_total else 0)


if __name__ == "__main__":
    main()
