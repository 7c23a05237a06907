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


STRUCTS = ("kp_str", "kp_label", "kp_requirement", "kp_cluster_affinity", "kp_affinity_term", "kp_toleration",
           "kp_taint", "kp_spread_constraint", "kp_static_weight", "kp_resource", "kp_target_cluster", "kp_binding",
           "kp_api_enablement", "kp_model_range", "kp_resource_model", "kp_allocatable_modeling", "kp_cluster",
           "kp_options", "kp_results", "kp_affinity_results", "kp_stage_times", "kp_component",
           "kp_kernel_time")


def test_abi_version_and_struct_sizes(tmp_path):
    """The ctypes mirrors (karmada_amd/api.py) have the C layout of every struct the
    header declares: sizes compiled from the header itself with the host compiler."""
    import subprocess
    L = engine.load_library()
    assert L.kp_abi_version() == engine.KP_ABI_VERSION
    src = tmp_path / "sizes.c"
    src.write_text('#include <stdio.h>\n#include "kp/kp_api.h"\nint main(void) {\n' +
                   "".join(f'  printf("%zu\\n", sizeof({n}));\n' for n in STRUCTS) + "  return 0;\n}\n")
    exe = tmp_path / "sizes"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)])
    sizes = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    for n, sz in zip(STRUCTS, sizes):
        assert C.sizeof(getattr(api, n)) == sz, n


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
