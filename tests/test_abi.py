"""CPU checks of the drop-in boundary: libkp.so loads and exports exactly the
entry points include/kp/kp_api.h declares (no compute calls: no GPU here)."""
import ctypes as C
import os
import re

from karmada_amd import api, engine, synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "kp", "kp_api.h")


def declared():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w ]+?\**\s*\b(kp_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_entry_points():
    names = declared()
    assert set(names) == set(engine.EXPORTS), names


def test_library_exports_every_declared_symbol():
    L = C.CDLL(engine.LIB_PATH)
    missing = [n for n in declared() if not hasattr(L, n)]
    assert not missing, missing


def test_abi_version_and_struct_sizes():
    L = engine.load_library()
    assert L.kp_abi_version() == engine.KP_ABI_VERSION
    # ctypes mirrors must match the C layout (x86-64 SysV)
    assert C.sizeof(api.kp_str) == 16
    assert C.sizeof(api.kp_results) == 64
    assert C.sizeof(api.kp_stage_times) == 64


def test_engine_create_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        return
    L = engine.load_library()
    h = C.c_void_p()
    assert L.kp_engine_create(0, C.byref(h)) == engine.KP_EDEVICE


def test_synth_ranges_are_slices_of_the_universe():
    whole = synth.Universe(6, 5, 40, 0, 300)
    part = synth.Universe(6, 5, 40, 100, 200)
    for i in range(100):
        a, b = whole.bindings[100 + i], part.bindings[i]
        assert C.string_at(a.uid.ptr, a.uid.len) == C.string_at(b.uid.ptr, b.uid.len)
        assert a.replicas == b.replicas and a.n_clusters == b.n_clusters
