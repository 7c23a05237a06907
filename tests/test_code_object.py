"""The built gfx950 code objects (karmada_amd/libkp.so) carry no kernel with a
dynamic call stack.

Round 4 root cause of the config 8 seed 6 divergence: the serial
Go pdqsort emulation (kp_algo.h pdqsort_go) recursed, which marks every kernel that
reaches it `.uses_dynamic_stack: true`; the runtime sizes such a kernel's scratch
from the static frame only, so thread 0 of k_slow (the serial emulation, deepest
stack) overran into the next wave's scratch and corrupted threads 64-65's spills.
Five kernels were affected (k_slow, k_select_cluster(_wide), k_region_b(_wide)).

The check reads the AMDGPU HSA metadata (msgpack) embedded in the offload bundle
of the shared library: every kernel map holds `.name` followed (keys sorted) by
`.uses_dynamic_stack` <bool>. Runs on CPU against the library the GPU box loads.
"""
import os
import re

import pytest

from karmada_amd.engine import PKG

LIB = os.path.join(PKG, "libkp.so")
KEY = b".uses_dynamic_stack"


def kernel_stack_flags(blob):
    out = []
    for m in re.finditer(re.escape(KEY), blob):
        flag = blob[m.end()]
        assert flag in (0xC2, 0xC3), "unexpected msgpack value after .uses_dynamic_stack"
        i = blob.rfind(b".name", 0, m.start())
        n = blob[i + 5]
        name = blob[i + 6:i + 6 + (n & 0x1F)] if 0xA0 <= n <= 0xBF else blob[i + 7:i + 7 + blob[i + 6]]
        out.append((name.decode(errors="replace"), flag == 0xC3))
    return out


def gpu_libraries():
    """Every gfx950 library in the package: libkp.so, the test-only device self-tests
    and any diagnostic variant (libkp_<name>.so; the round-4 illegal access in
    gpurun_out/d8m.log came from such a variant, built before the fix)."""
    import glob
    return sorted(p for p in glob.glob(os.path.join(PKG, "libkp*.so"))
                  if os.path.basename(p) not in ("libkp_cpusim.so", "libkpsynth.so"))


@pytest.mark.parametrize("lib", gpu_libraries(), ids=os.path.basename)
def test_no_dynamic_stack_in_any_gpu_library(lib):
    flags = kernel_stack_flags(open(lib, "rb").read())
    assert flags, f"{lib}: no kernel metadata found"
    bad = sorted(n for n, dyn in flags if dyn)
    assert not bad, f"{os.path.basename(lib)}: kernels with a dynamic (unsized) call stack: {bad}"


@pytest.mark.skipif(not os.path.exists(LIB), reason="libkp.so not built")
def test_no_kernel_uses_a_dynamic_stack():
    blob = open(LIB, "rb").read()
    flags = kernel_stack_flags(blob)
    names = {n for n, _ in flags}
    # every translation unit's code object was seen (sanity of the scan)
    for k in ("k_slow", "k_select_top", "k_region_b", "k_select_cluster", "k_filter"):
        assert any(n.startswith(k) for n in names), (k, sorted(names))
    bad = sorted(n for n, dyn in flags if dyn)
    assert not bad, f"kernels with a dynamic (unsized) call stack: {bad}"


def test_scan_reads_both_flags():
    """The scanner on a synthetic metadata fragment (fixstr and str8 names)."""
    frag = (b"\xa5.name\xa6k_slow\xbb.private_segment_fixed_size\xcd\x05p" + b"\xb3" + KEY + b"\xc3" +
            b"\xa5.name\xd9\x21" + b"k" * 0x21 + b"\xb3" + KEY + b"\xc2")
    assert kernel_stack_flags(frag) == [("k_slow", True), ("k" * 0x21, False)]
