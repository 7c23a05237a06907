"""Device self-test of the workgroup primitives (kp_blk.h GpuBlk: DPP wave
reductions/scans, double-buffered cross-wave scratch, histogram search) against
host results, for every workgroup size the kernels launch with."""
import ctypes as C
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "karmada_amd", "libkp_blktest.so")


@pytest.mark.gpu
@pytest.mark.parametrize("nth", [64, 128, 256, 512, 1024])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_block_primitives(nth, seed):
    lib = C.CDLL(LIB)
    lib.kp_blk_selftest.restype = C.c_int
    lib.kp_blk_selftest.argtypes = [C.c_int, C.c_int, C.c_uint64, C.c_char_p, C.c_int]
    msg = C.create_string_buffer(256)
    bad = lib.kp_blk_selftest(nth, 37, seed, msg, 256)
    assert bad == 0, msg.value.decode()


@pytest.mark.gpu
@pytest.mark.parametrize("nth", [64, 256, 512])
def test_sort_tcl_wave_form_on_device(nth):
    """Go sort.Sort over TargetClustersList emulated by one wave64 (kp_pdq.h)
    gives the oracle's permutation, including the order of equal replicas."""
    import oracle_lib as O
    import pdq_cases
    lib = C.CDLL(LIB)
    lib.kp_pdq_selftest.restype = C.c_int
    lib.kp_pdq_selftest.argtypes = [C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.c_int, C.c_int,
                                    C.POINTER(C.c_uint32), C.c_char_p, C.c_int]
    L = O.lib()
    L.kpo_sort_target_clusters.argtypes = [C.POINTER(C.c_int32), C.POINTER(C.c_uint32), C.c_uint32]
    lists = []
    for seed in range(3):
        lists += [(n, kind, reps) for n, kind, reps in pdq_cases.cases(seed)]
    offs, flat = [0], []
    for _, _, reps in lists:
        flat += reps
        offs.append(len(flat))
    reps_c = (C.c_int32 * max(1, len(flat)))(*flat)
    offs_c = (C.c_int32 * len(offs))(*offs)
    out = (C.c_uint32 * max(1, len(flat)))()
    msg = C.create_string_buffer(256)
    declined = lib.kp_pdq_selftest(reps_c, offs_c, len(lists), nth, out, msg, 256)
    assert declined == 0, msg.value.decode()
    for j, (n, kind, reps) in enumerate(lists):
        ids = (C.c_uint32 * max(1, n))(*range(n))
        rr = (C.c_int32 * max(1, n))(*reps)
        L.kpo_sort_target_clusters(rr, ids, n)
        want = [ids[i] for i in range(n)]
        got = [out[offs[j] + i] for i in range(n)]
        assert got == want, (n, kind)


@pytest.mark.gpu
def test_webster_reg_on_device():
    """webster_reg (kp_select.h): AllocateWebsterSeats with one party per lane of one
    wave, in registers (k_select_top's subsets of <= 64 candidates), gives the oracle's
    seats (webstermethod.go:112-161, the heap's tie-breaker both name orders) on seeded
    lists: tied votes, one party, zero votes, large and small seat counts."""
    import random
    import oracle_lib as O
    from karmada_amd import api
    lib = C.CDLL(LIB)
    lib.kp_webster_reg_selftest.restype = C.c_int
    lib.kp_webster_reg_selftest.argtypes = [C.POINTER(C.c_int64), C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                            C.POINTER(C.c_int32), C.c_int, C.POINTER(C.c_int32), C.c_char_p,
                                            C.c_int]
    L = O.lib()
    rng = random.Random(7)
    cases = []
    while len(cases) < 3000:
        n = rng.choice([1, 2, 3, 5, 8, 13, 31, 32, 33, 50, 63, 64])
        kind = rng.randrange(5)
        if kind == 0:
            votes = [rng.randint(0, 20) for _ in range(n)]  # many ties
        elif kind == 1:
            votes = [rng.choice([7, 7, 7, 21, 35]) for _ in range(n)]
        elif kind == 2:
            votes = [rng.randint(1, 5000) for _ in range(n)]
        elif kind == 3:
            votes = [rng.randint(0, 2**31 // 64 - 1) for _ in range(n)]
        else:
            votes = [rng.choice([0, 1, 3, 9, 27, 81, 243]) for _ in range(n)]
        if sum(votes) == 0:
            continue  # Dispenser returns before Webster (binding.go:98-101)
        N = rng.choice([1, 2, 3, 7, 10, 33, 64, 100, 257, 1000, 50000])
        cases.append((votes, N, rng.choice([0, 1])))
    offs, flat = [0], []
    for votes, _, _ in cases:
        flat += votes
        offs.append(len(flat))
    nl = len(cases)
    out = (C.c_int32 * len(flat))()
    msg = C.create_string_buffer(256)
    declined = lib.kp_webster_reg_selftest((C.c_int64 * len(flat))(*flat), (C.c_int32 * len(offs))(*offs),
                                           (C.c_int32 * nl)(*[c[1] for c in cases]),
                                           (C.c_int32 * nl)(*[c[2] for c in cases]), nl, out, msg, 256)
    assert declined == 0, msg.value.decode()
    bad = 0
    for j, (votes, N, desc) in enumerate(cases):
        n = len(votes)
        w = api.World()
        names, _ = w.arr(api.kp_str, [w.s("m%03d" % i) for i in range(n)])
        want = (C.c_int32 * n)()
        L.kpo_allocate_webster(N, names, (C.c_int64 * n)(*votes), n, None, None, 0, 2 if desc else 1,
                               api.kp_str(None, 0), want, n)
        got = [out[offs[j] + i] for i in range(n)]
        if got != list(want):
            bad += 1
            assert bad < 1, (votes, N, desc, got, list(want))
