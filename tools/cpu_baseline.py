"""CPU baseline of the reference's algorithm (the oracle's restatement, test
infrastructure) for BASELINE.md §3: config 1 in full (FAITHFUL mode: the literal
loops, per-binding snapshot deep copy) at 1 thread and at every CPU this process
may use, bounded REFSHAPE samples of configs 2-5, and config 3's FAITHFUL
per-pair sample: seeded (binding, cluster) pairs through the
literal first-fit loop of the resource-model estimator, extrapolated to a
per-binding cost. One JSON line.

    python tools/cpu_baseline.py [--budget SECONDS]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from bench import cpu_threads  # noqa: E402
from karmada_amd import api, synth  # noqa: E402
import oracle_lib as O  # noqa: E402


def timed(u, n, mode, th):
    ba, _ = u.binding_slice(0, n)
    t0 = time.perf_counter()
    O.schedule_c(u.clusters, u.n_clusters, ba, n, api.options(), mode, th)
    return time.perf_counter() - t0


def sample(u, mode, th, budget):
    n = 16
    while True:
        n = min(n, u.n_bindings)
        dt = timed(u, n, mode, th)
        if dt >= budget or n >= u.n_bindings:
            return n, dt
        n *= 2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--budget", type=float, default=8.0)
    args = ap.parse_args()
    T = cpu_threads()
    out = {"cores": T, "os_cpu_count": os.cpu_count(), "configs": {}}
    u = synth.Universe(1, 1, synth.CONFIGS[1][0], 0, synth.CONFIGS[1][1])  # config 1: C=10, B=1000, seed 1
    for th in (1, T):
        dt = timed(u, u.n_bindings, O.FAITHFUL, th)
        out["configs"].setdefault("1", {})[f"faithful_{th}t"] = {"bindings": u.n_bindings, "s": round(dt, 3),
                                                                   "per_s": round(u.n_bindings / dt, 1)}
    for cfg in (2, 3, 4, 5):
        C_, B_ = synth.CONFIGS[cfg]
        u = synth.Universe(cfg, cfg, C_, 0, min(B_, 4096))
        for th in (1, T):
            n, dt = sample(u, O.REFSHAPE, th, args.budget)
            out["configs"].setdefault(str(cfg), {})[f"refshape_{th}t"] = {"bindings": n, "s": round(dt, 3),
                                                                            "per_s": round(n / dt, 2)}
            print(f"config {cfg} {th}t: {n} bindings in {dt:.2f} s", file=sys.stderr, flush=True)
    out["configs"]["3"]["faithful_pairs_1t"] = faithful_pairs(args.budget)
    print(json.dumps(out))


def faithful_pairs(budget):
    """Config 3, 1 thread: seeded (binding, cluster) pairs; each pair's filter
    (kpo_filter) decides whether the reference would estimate it, and the feasible
    ones run GeneralEstimator.maxAvailableReplicas in FAITHFUL mode (the literal FF
    loop over the model-grade nodes). bindings/s = 1 / (C x feasible fraction x
    mean estimate time): the estimator alone, so an upper bound on the reference's
    rate at this config."""
    import ctypes as C
    import random
    L = O.lib()
    C_, B_ = synth.CONFIGS[3]
    u = synth.Universe(3, 3, C_, 0, 2048)
    opts = api.options()
    r = random.Random(3)
    t_est = 0.0
    n_pairs = n_feas = 0
    t_end = time.perf_counter() + budget
    while time.perf_counter() < t_end and n_pairs < 10000:
        b = r.randrange(u.n_bindings)
        c = r.randrange(u.n_clusters)
        cp = C.pointer(u.clusters[c])
        bp = C.pointer(u.bindings[b])
        n_pairs += 1
        if L.kpo_filter(cp, bp, C.byref(opts)) != 0:
            continue
        n_feas += 1
        t0 = time.perf_counter()
        L.kpo_max_available_replicas(cp, bp, C.byref(opts), O.FAITHFUL)
        t_est += time.perf_counter() - t0
    per = t_est / max(1, n_feas)
    frac = n_feas / max(1, n_pairs)
    return {"pairs": n_pairs, "feasible": n_feas, "s": round(t_est, 3), "per_pair_us": round(per * 1e6, 2),
            "per_s": round(1.0 / (C_ * frac * per), 4) if per > 0 and frac > 0 else None}


if __name__ == "__main__":
    main()
