"""Transcribes the pkg/util/binding_test.go tables the placement path relies on into
tests/golden/util_binding.json (round 3): TestGetSumOfReplicas (:258; the int32 sum
of hazard H5), TestMergeTargetClusters (:332) and TestRescheduleRequired (:443;
metav1.Now() and Now()-1m become the integer times 2000 and 1000); and the
runtime.Registry tables (framework/runtime/registry_test.go) that the `--plugins`
mirror (kp_options.enabled_plugins, karmada_amd/plugins.py) follows.
Development-container only (reads /root/reference); the JSON it writes is
committed and is all the test suite reads.

    python tests/golden/make_golden_r3.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from goconv import Conv  # noqa: E402
from gotables import table  # noqa: E402

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
PATH = "pkg/util/binding_test.go"


def main():
    with open(os.path.join(REF, PATH), encoding="utf-8") as f:
        src = f.read()
    cv = Conv({"nil": None, "&currentTime": 2000, "&previousTime": 1000, "currentTime": 2000, "previousTime": 1000})
    out = {"source": [], "sum": [], "merge": [], "reschedule": []}
    rows, line = table(src, "TestGetSumOfReplicas")
    out["source"].append("%s:%d (TestGetSumOfReplicas)" % (PATH, line))
    for r in rows:
        out["sum"].append({"name": cv.ev(r.get("name")), "clusters": cv.targets(r.get("clusters")),
                           "expected": cv.ev(r.get("expected"))})
    rows, line = table(src, "TestMergeTargetClusters")
    out["source"].append("%s:%d (TestMergeTargetClusters)" % (PATH, line))
    for r in rows:
        out["merge"].append({"name": cv.ev(r.get("name")), "old": cv.targets(r.get("old")),
                             "new": cv.targets(r.get("new")), "expected": cv.targets(r.get("expected"))})
    rows, line = table(src, "TestRescheduleRequired")
    out["source"].append("%s:%d (TestRescheduleRequired; Now() = 2000, Now()-1m = 1000)" % (PATH, line))

    def t(v):
        if v is None:
            return None
        v = cv.ev(v)
        return None if v in (None, "nil") else v
    for r in rows:
        out["reschedule"].append({"name": cv.ev(r.get("name")), "rescheduleTriggeredAt": t(r.get("rescheduleTriggeredAt")),
                                  "lastScheduledTime": t(r.get("lastScheduledTime")), "want": cv.ev(r.get("want"))})
    # runtime.Registry (pkg/scheduler/framework/runtime/registry_test.go): its rows hold
    # only names and string lists, read field by field (the Registry-typed field `r`
    # is the table's fixed registry of `plugins`)
    import re
    rpath = "pkg/scheduler/framework/runtime/registry_test.go"
    with open(os.path.join(REF, rpath), encoding="utf-8") as f:
        rsrc = f.read()
    registered = re.findall(r'"([^"]*)"', re.search(r"plugins := \[\]string\{([^}]*)\}", rsrc).group(1))

    def rows_of(func):
        body_start = rsrc.index("func %s(" % func)
        body = rsrc[body_start:rsrc.index("\nfunc ", body_start + 1)]
        line = rsrc[:body_start].count("\n") + 1
        out_rows = []
        for blk in re.split(r"\n\t\t\{\n", body)[1:]:
            row = {}
            for k, v in re.findall(r"(\w+):\s+(\[\]string\{[^}]*\}|nil|\"[^\"]*\"|true|false|r),", blk):
                if v.startswith("[]string"):
                    row[k] = re.findall(r'"([^"]*)"', v)
                elif v == "nil":
                    row[k] = []
                elif v in ("true", "false"):
                    row[k] = v == "true"
                elif v.startswith('"'):
                    row[k] = v[1:-1]
            if "name" in row:
                out_rows.append(row)
        return out_rows, line
    reg = {"source": [], "filter": [], "register": [], "unregister": []}
    rows, line = rows_of("TestRegistry_Filter")
    reg["source"].append("%s:%d (TestRegistry_Filter)" % (rpath, line))
    for r in rows:
        reg["filter"].append({"name": r["name"], "registered": registered, "curPlugins": r["curPlugins"],
                              "expectedPlugins": r["expectedPlugins"]})
    for fn, key, arg in (("TestRegistry_Register", "register", "registeringPlugin"),
                         ("TestRegistry_Unregister", "unregister", "removingPlugin")):
        rows, line = rows_of(fn)
        reg["source"].append("%s:%d (%s)" % (rpath, line, fn))
        for r in rows:
            reg[key].append({"name": r["name"], "initialPlugins": r.get("initialPlugins", []), "plugin": r[arg],
                             "wantErr": r["wantErr"], "expectedPlugins": r["expectedPlugins"]})
    out["registry"] = reg
    with open(os.path.join(OUT, "util_binding.json"), "w") as f:
        json.dump(out, f, indent=1)
    print({k: len(v) for k, v in out.items()})


if __name__ == "__main__":
    main()
