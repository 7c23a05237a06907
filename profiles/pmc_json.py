"""Per-kernel, per-launch PMC summary (profiles/rNN_pmc_config<N>.json, the format bench.py's
load_pmc reads) from the rocprofv3 passes of tools/gpu/prof_pmc.sh under gpurun_out/pmc_<tag>/.

    python profiles/pmc_json.py gpurun_out/pmc_<tag> <out.json> "<command description>"

HBM bytes per launch = FETCH_SIZE x 2 (gfx950 under-counts FETCH_SIZE by 2x,
MI355X_MICROARCH.md) + WRITE_SIZE, both reported by rocprofv3 in KB.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_table import load  # noqa: E402


def main():
    src, out, cmd = sys.argv[1], sys.argv[2], sys.argv[3]
    ks = {}
    for k, cs in sorted(load(src).items()):
        e = dict(cs)
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            e["fetch_bytes_x2"] = cs["FETCH_SIZE"] * 1024 * 2
            e["write_bytes"] = cs["WRITE_SIZE"] * 1024
            e["hbm_bytes"] = e["fetch_bytes_x2"] + e["write_bytes"]
        if "TCC_HIT_sum" in cs and "TCC_MISS_sum" in cs:
            e["l2_hit_rate"] = cs["TCC_HIT_sum"] / max(1.0, cs["TCC_HIT_sum"] + cs["TCC_MISS_sum"])
        if "SQ_INSTS_VALU" in cs:
            e["valu_insts"] = cs["SQ_INSTS_VALU"]
        if "SQ_WAIT_ANY" in cs and "SQ_WAVE_CYCLES" in cs:
            e["wait_share"] = cs["SQ_WAIT_ANY"] / max(1.0, cs["SQ_WAVE_CYCLES"])
        ks[k] = e
    with open(out, "w") as f:
        json.dump({"command": cmd, "source": src, "kernels": ks}, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
