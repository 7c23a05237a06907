"""Per-kernel, per-launch PMC table from gpurun_out/pmc_<tag>/p*/ (rocprofv3 csv)."""
import collections
import csv
import glob
import os
import sys


def load(d):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "p*", "*", "*_counter_collection.csv")) + glob.glob(
            os.path.join(d, "p*", "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            per[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items() if not k.startswith("__amd")}


if __name__ == "__main__":
    for k, cs in sorted(load(sys.argv[1]).items()):
        print(k)
        for c, v in sorted(cs.items()):
            print(f"  {c:40s} {v:14.4g}")
