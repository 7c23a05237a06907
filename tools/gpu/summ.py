"""Summary of bench.py JSON lines: python tools/gpu/summ.py file... (rate, step, serial, e2e,
parity, the five slowest kernels, every launch with 0 units)."""
import json
import sys
for f in sys.argv[1:]:
    try:
        d = json.loads([x for x in open(f) if x.startswith("{")][-1])
    except Exception as ex:  # noqa: BLE001
        print(f, "no line:", ex)
        continue
    ks = sorted(d.get("kernels", []), key=lambda k: -k["ms"])
    print(f, d["config"]["workload"][:8], "value %.1fM" % (d["value"] / 1e6), "ms", d["ms_per_step"], "serial",
          d.get("serial_ms_per_step"), "e2e", d.get("end_to_end_value"), "parity", d.get("parity_checked"),
          d.get("parity_bad"))
    print("   top:", [(k["kernel"], k["ms"], k["units"]) for k in ks[:6]])
    print("   idle:", [(k["kernel"], k["ms"]) for k in ks if k["units"] == 0])
