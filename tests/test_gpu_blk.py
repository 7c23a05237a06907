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
