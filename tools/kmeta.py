"""Per-kernel resource metadata of the gfx950 code objects: LDS, private (scratch)
segment per lane, VGPR/AGPR counts and spills. Scratch traffic (spills, stack
arrays) is invisible in the source; this is the first place to look for it.

    python tools/kmeta.py karmada_amd/csrc/kernels_tu*.o
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def kernels(obj):
    with tempfile.TemporaryDirectory() as d:
        elf, fat = os.path.join(d, "co.elf"), os.path.join(d, "fat.bin")
        # a host object (hipcc -c) carries the offload bundle in its .hip_fatbin section
        r = subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(d, "x.o")],
                           capture_output=True)
        src = fat if r.returncode == 0 and os.path.exists(fat) else obj
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        f"--input={src}", f"--output={elf}", "--unbundle"], check=True, capture_output=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", elf], check=True, capture_output=True,
                               text=True).stdout
    out, cur, in_args = [], {}, False
    for line in notes.splitlines():
        m = re.match(r"(\s+)(- )?\.(\w+):\s*(\S*)", line)
        if not m:
            continue
        k, v = m.group(3), m.group(4)
        if k == "args":
            in_args = True
            continue
        if in_args and len(m.group(1)) > 6:
            continue
        in_args = False
        cur[k] = v
        if k == "wavefront_size":
            out.append(cur)
            cur = {}
    return [c for c in out if not c.get("name", "_").startswith("__")]


def main():
    seen = set()
    for obj in sys.argv[1:]:
        for c in kernels(obj):
            n = c.get("name")
            if n in seen:
                continue
            seen.add(n)
            print(f"{n:30s} lds={c.get('group_segment_fixed_size')} priv={c.get('private_segment_fixed_size')} "
                  f"vgpr={c.get('vgpr_count')} agpr={c.get('agpr_count')} vspill={c.get('vgpr_spill_count')} "
                  f"sspill={c.get('sgpr_spill_count')} dynstack={c.get('uses_dynamic_stack')}")


if __name__ == "__main__":
    main()
