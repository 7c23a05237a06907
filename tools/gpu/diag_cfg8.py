"""Round-4 diagnostic: repeated GPU runs of one seeded universe against the oracle,
printing for each differing binding its route inputs and the target-set difference.

    python tools/gpu/diag_cfg8.py <lib.so> config:seed:clusters:bindings passes [ENV=V ...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from karmada_amd import api, synth  # noqa: E402
from karmada_amd.engine import Batch, Engine, Snapshot  # noqa: E402
import oracle_lib as O  # noqa: E402


def s(x):
    return x.ptr[:x.len].decode() if x.len else ""


def main():
    lib, spec, passes = sys.argv[1], sys.argv[2], int(sys.argv[3])
    for kv in sys.argv[4:]:
        k, v = kv.split("=", 1)
        os.environ[k] = v
    cfg, seed, C_, B_ = (int(x) for x in spec.split(":"))
    e = Engine(0, lib_path=lib)
    u = synth.Universe(cfg, seed, C_, 0, B_)
    opts = api.options()
    no_oracle = os.environ.get("DIAG_NO_ORACLE") == "1"  # (stage counts only, e.g. KP_DEBUG_SLOW)
    want = None if no_oracle else O.schedule_c(u.clusters, u.n_clusters, u.bindings, u.n_bindings, opts, O.FAST, 8)
    snap = Snapshot.from_structs(e, u.clusters, u.n_clusters, u.names, opts)
    for p in range(passes):
        b = Batch(snap, structs=u.binding_slice(0, B_))
        got = b.schedule()
        t = e.stage_times()
        b.close()
        bad = [] if want is None else [i for i, (g, w) in enumerate(zip(got, want)) if g != w]
        print(f"pass {p}: {len(bad)} differ; n_slow {t.get('n_slow')} bits {t.get('bits')} top {t.get('n_top')}",
              flush=True)
        for i in bad[:12]:
            bd = u.bindings[i]
            g, w = got[i], want[i]
            gt, wt = dict(g["targets"]), dict(w["targets"])
            miss = sorted(set(wt) - set(gt))
            extra = sorted(set(gt) - set(wt))
            diffv = sorted(c for c in set(gt) & set(wt) if gt[c] != wt[c])
            print(f"  b{i}: rep {bd.replicas} {s(bd.replica_scheduling_type)}/{s(bd.replica_division_preference)}"
                  f" dyn={s(bd.dynamic_weight)} sw={bd.n_static_weights} tgt={bd.n_clusters} spread={bd.n_spread_constraints}"
                  f" | got st{g['status']} e{g['err']} a{g['arg']} n{len(gt)} sum{sum(gt.values())}"
                  f" | want st{w['status']} e{w['err']} a{w['arg']} n{len(wt)} sum{sum(wt.values())}"
                  f" | missing {miss[:8]} extra {extra[:8]} changed {len(diffv)} {diffv[:6]}", flush=True)
    snap.close()
    e.close()


if __name__ == "__main__":
    main()
