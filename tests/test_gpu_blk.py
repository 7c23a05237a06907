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
