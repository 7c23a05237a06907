"""Per-kernel, per-launch PMC summary (the JSON bench.py reads for its roofline) from
the rocprofv3 passes of prof_pmc.sh: gpurun_out/pmc_<tag>/p*/.

usage: python profiles/pmc_r02.py gpurun_out/pmc_<tag> profiles/r0N_pmc_config<N>.json "<bench command>"

hbm_bytes = FETCH_SIZE*2 + WRITE_SIZE per launch, in bytes: rocprofv3 reports both in
KiB, and on gfx950 FETCH_SIZE counts half the bytes of wide coalesced reads
(MI355X_MICROARCH.md, HBM), so it is doubled. valu_insts = SQ_INSTS_VALU (wave
instructions) per launch.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_table import load  # noqa: E402


def main():
    src, out = sys.argv[1], sys.argv[2]
    cmd = sys.argv[3] if len(sys.argv) > 3 else ""
    ks = {}
    for k, cs in sorted(load(src).items()):
        e = {c: v for c, v in cs.items()}
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            e["fetch_bytes_x2"] = 2 * 1024 * cs["FETCH_SIZE"]
            e["write_bytes"] = 1024 * cs["WRITE_SIZE"]
            e["hbm_bytes"] = e["fetch_bytes_x2"] + e["write_bytes"]
        if "SQ_INSTS_VALU" in cs:
            e["valu_insts"] = cs["SQ_INSTS_VALU"]
        if "SQ_WAVE_CYCLES" in cs and "SQ_WAIT_ANY" in cs:
            e["wait_share"] = cs["SQ_WAIT_ANY"] / max(1.0, cs["SQ_WAVE_CYCLES"])
        if "TCC_HIT_sum" in cs and "TCC_MISS_sum" in cs:
            e["l2_hit_rate"] = cs["TCC_HIT_sum"] / max(1.0, cs["TCC_HIT_sum"] + cs["TCC_MISS_sum"])
        ks[k] = e
    with open(out, "w") as f:
        json.dump({"command": cmd, "source": src, "kernels": ks}, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
