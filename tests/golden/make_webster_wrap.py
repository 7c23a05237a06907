"""Generates tests/golden/webster_wrap.json: AllocateWebsterSeats (pkg/util/helper/
webstermethod.go:112-161) where Go's int32 `2*Seats+1` wraps (seat counts past 2^30)
or votes are zero/negative (SURVEY hazard H5), answered by the oracle's LITERAL heap
loop (one pop per seat, up to 2^31 pops per case: minutes). The reference has no
table for these sizes; the literal loop restates webstermethod.go:57-85,112-161
line by line and is itself pinned by TestAllocateWebsterSeats (tests/golden/
webster.json). Run from the repo root: python tests/golden/make_webster_wrap.py"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from karmada_amd import api  # noqa: E402
import oracle_lib as O  # noqa: E402

# (votes, seats, tie_mode: 1 = names ascending (even UID hash), 2 = descending (odd))
CASES = [
    ([1000000000, 0, 0], 2**30 + 7, 1),
    ([1000000000, 0, 0], 2**30 + 8, 2),
    ([2000000000, 1], 2**30 + 100000, 1),
    ([7, 1900000000, 3, 0], 2**30 + 12345, 2),
    ([-5, -3, -9], 100, 1),
    ([-5, 0, -3, 0], 1001, 2),
    ([1200000000, -5, -3], 2**31 - 1, 1),
    ([1500000000, 0], 2**31 - 1, 1),
    ([2000000000, 1000000000], 2**31 - 1, 2),
    ([400000000, 400000000, 400000000, 0], 2**31 - 1, 1),
    ([3, 1200000000], 2**30 + 1000, 1),
]


def literal(votes, n_seats, tie):
    L = O.lib()
    L.kpo_set_webster_fast.argtypes = [C.c_int]
    L.kpo_set_webster_fast(0)
    w = api.World()
    n = len(votes)
    names, _ = w.arr(api.kp_str, [w.s(f"member{i + 1}") for i in range(n)])
    vv = (C.c_int64 * n)(*votes)
    out = (C.c_int32 * n)()
    L.kpo_allocate_webster(n_seats, names, vv, n, None, None, 0, tie, api.kp_str(None, 0), out, n)
    return list(out)


def main():
    cases = []
    for votes, n_seats, tie in CASES:
        t0 = time.time()
        seats = literal(votes, n_seats, tie)
        print(votes, n_seats, tie, seats, f"{time.time() - t0:.0f}s", flush=True)
        cases.append({"votes": votes, "seats": n_seats, "tie_mode": tie,
                      "names": [f"member{i + 1}" for i in range(len(votes))], "want": seats})
    path = os.path.join(ROOT, "tests", "golden", "webster_wrap.json")
    with open(path, "w") as f:
        json.dump({"source": "oracle literal heap loop (webstermethod.go:57-85,112-161), "
                             "tests/golden/make_webster_wrap.py", "cases": cases}, f, indent=1)


if __name__ == "__main__":
    main()
