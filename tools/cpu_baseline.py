"""CPU baseline of the reference's algorithm (the oracle's restatement, test
infrastructure) for BASELINE.md §3: config 1 in full (FAITHFUL mode: the literal
loops, per-binding snapshot deep copy) at 1 thread and at every CPU this process
may use, and bounded REFSHAPE samples of configs 2 and 3. One JSON line.

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
    for cfg in (2, 3):
        C_, B_ = synth.CONFIGS[cfg]
        u = synth.Universe(cfg, cfg, C_, 0, min(B_, 4096))
        for th in (1, T):
            n, dt = sample(u, O.REFSHAPE, th, args.budget)
            out["configs"].setdefault(str(cfg), {})[f"refshape_{th}t"] = {"bindings": n, "s": round(dt, 3),
                                                                            "per_s": round(n / dt, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
