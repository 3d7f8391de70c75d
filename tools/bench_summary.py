"""One-line summary of a bench.py JSON output file: value, ms, rooflines, top kernels."""
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(d["value"], "Mpts/s", d["ms_per_step"], "ms", d["dtype"])
r = d.get("roofline") or {}
print("roofline", r.get("kernel"), r.get("bound"), r.get("achieved"), r.get("frac"), "traffic", r.get("traffic"))
for k, v in (d.get("rooflines") or {}).items():
    print(" ", k, v.get("achieved"), v.get("frac"), v.get("ms") or v.get("us"), v.get("roofline_frac", ""))
for k, v in list((d.get("kernels") or {}).items())[:int(sys.argv[2]) if len(sys.argv) > 2 else 0]:
    print("   ", v, k)
