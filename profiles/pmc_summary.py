"""Summarise rocprofv3 PMC passes (gpurun_out/prof_*) into per-kernel, per-launch figures.

Usage: python profiles/pmc_summary.py <gpurun_out dir> <out.json> [--traffic profiles/traffic_config3.json]

HBM traffic per launch = FETCH_SIZE + WRITE_SIZE (rocprofv3 reports kilobytes). On gfx950
FETCH_SIZE under-counts wide coalesced streaming reads by 2x (MI355X_MICROARCH.md, HBM);
the pair kernel's reads are narrow L2-served column loads, so the raw value is kept and
the 2x-corrected one is reported beside it as an upper bound.
"""
import collections
import csv
import glob
import json
import os
import sys


def load(d):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "prof_*", "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0]
            per[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items()}


def main():
    src, out = sys.argv[1], sys.argv[2]
    traffic_path = sys.argv[sys.argv.index("--traffic") + 1] if "--traffic" in sys.argv else None
    per = load(src)
    res = {}
    for k, cs in sorted(per.items()):
        if k.startswith("__amd"):
            continue
        e = dict(cs)
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            f, w = cs["FETCH_SIZE"] * 1024, cs["WRITE_SIZE"] * 1024
            e["hbm_bytes_per_launch"] = f + w
            e["hbm_bytes_per_launch_fetch2x"] = 2 * f + w
        if "TCC_HIT_sum" in cs and "TCC_MISS_sum" in cs:
            e["l2_hit_rate"] = cs["TCC_HIT_sum"] / max(1.0, cs["TCC_HIT_sum"] + cs["TCC_MISS_sum"])
        if "SQ_INSTS_VALU" in cs and "SQ_WAVES" in cs:
            e["valu_insts_per_wave"] = cs["SQ_INSTS_VALU"] / cs["SQ_WAVES"]
        if all(x in cs for x in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")):
            tot = cs["SQ_WAIT_ANY"] + cs["SQ_WAIT_INST_ANY"] + cs["SQ_ACTIVE_INST_ANY"]
            e["wave_time_share"] = {"waiting": cs["SQ_WAIT_ANY"] / tot, "issue_stall": cs["SQ_WAIT_INST_ANY"] / tot,
                                    "active": cs["SQ_ACTIVE_INST_ANY"] / tot}
        res[k] = e
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    pair = [k for k in res if k.startswith("k_pair") and "hbm_bytes_per_launch" in res[k]]
    kp = max(pair, key=lambda k: res[k].get("SQ_WAVES", 0)) if pair else "k_pair"  # the instance the bench ran
    if traffic_path and kp in res and "hbm_bytes_per_launch" in res[kp]:
        with open(traffic_path, "w") as fh:
            json.dump({"k_pair_bytes_per_launch": res[kp]["hbm_bytes_per_launch"],
                       "k_pair_valu_per_launch": res[kp].get("SQ_INSTS_VALU"),
                       "kernel": kp,
                       "source": os.path.basename(out),
                       "note": "FETCH_SIZE+WRITE_SIZE and SQ_INSTS_VALU per pair-kernel launch, "
                               "rocprofv3 separate --pmc passes"}, fh, indent=1)
    print(json.dumps({k: {kk: v for kk, v in e.items() if not kk.startswith("SQ_")} for k, e in res.items()}, indent=1))


if __name__ == "__main__":
    main()
