"""Effective shader clock per kernel label from a rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace pass
(MI355X_MICROARCH.md "DVFS give-back": GRBM_GUI_ACTIVE is summed over the 8 XCDs, so the clock is
GRBM_GUI_ACTIVE / 8 / kernel wall time; it reads high on dispatches shorter than ~0.3 ms).

    python tools/pmc_clock.py <pmc dir> <out.json>
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import label  # noqa: E402


def main(d, out):
    ctr = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                ctr[r["Dispatch_Id"]] = (r["Kernel_Name"], float(r["Counter_Value"]))
    dur = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[r["Dispatch_Id"]] = (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-9
    acc = defaultdict(lambda: [0.0, 0.0, 0])
    for did, (name, v) in ctr.items():
        if did in dur and dur[did] > 0:
            a = acc[label(name)]
            a[0] += v / 8.0
            a[1] += dur[did]
            a[2] += 1
    res = {k: {"clock_ghz": round(c / t / 1e9, 3), "dispatches": n, "avg_us": round(t / n * 1e6, 1)}
           for k, (c, t, n) in acc.items()}
    with open(out, "w") as fh:
        json.dump({"source": "rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace, eager bench steps: clock = "
                             "sum(GRBM_GUI_ACTIVE / 8) / sum(kernel wall time) per label (reads high below ~0.3 ms)",
                   "kernels": res}, fh, indent=1, sort_keys=True)
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]["avg_us"] * kv[1]["dispatches"])[:12]:
        print(f"{k:60s} {v['clock_ghz']:6.3f} GHz  {v['avg_us']:8.1f} us x {v['dispatches']}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
