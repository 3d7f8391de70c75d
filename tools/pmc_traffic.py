"""HBM traffic per launch, by bench kernel label, from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

    python tools/pmc_traffic.py <pmc dir> <out.json>

MI355X_MICROARCH.md (HBM section): on gfx950 FETCH_SIZE reports half the bytes of a
wide streaming read, WRITE_SIZE the bytes of 16-B-per-lane stores; both in KB.  So
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024   per dispatch.
Labels follow bench.py's `kernels` keys (ops.gemm_kernel_label / kernel names).
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

EPI = {"0": "plain", "1": "res_f32", "2": "res_bf16", "3": "res2", "4": "convT", "5": "q8", "6": "ln_fold"}


def label(name: str) -> str:
    n = re.sub(r"^void ", "", name.split("(")[0].strip())
    n = re.sub(r"\b[A-Za-z_]\w*::", "", n)
    # k_gemm_p<BM, CONV, RELU_A, EPI[, BN, F8]> -> the bench labels (gemm.hip plan_name / plan8_name)
    m = re.match(r"k_gemm_p<(\d+), (\w+), (\w+), (\d+)(?:, (\d+), (\w+))?>", n)
    if m:
        if m[6] == "true":
            return f"k_gemm_f8<{m[5]}, {m[2]}, {m[3]}, {EPI.get(m[4], m[4])}>"
        return f"k_gemm_p<{m[1]}, {m[2]}, {m[3]}, {EPI.get(m[4], m[4])}>"
    if n.startswith("k_attention"):
        return "k_attention"
    return n


def main(d, out, steps=2):
    """steps: eager bench steps per pass (tools/gpu.sh profile runs `--steps 1 --no-graph`, which
    steps once before the timed step: 2), so per-step totals are the pass sums / steps."""
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            acc[label(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, cs in acc.items():
        if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        fetch = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"])
        write = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"])
        res[k] = {"fetch_size_kb": round(fetch, 1), "write_size_kb": round(write, 1),
                  "dispatches": len(cs["FETCH_SIZE"]),
                  "hbm_bytes_per_launch": round((2 * fetch + write) * 1024),
                  # every dispatch of the label in one step (e.g. a GEMM call's main + tail launch)
                  "hbm_bytes_per_step": round((2 * sum(cs["FETCH_SIZE"]) + sum(cs["WRITE_SIZE"])) * 1024 / steps)}
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import kernels_sha16
    with open(out, "w") as fh:
        json.dump({"kernels_sha16": kernels_sha16(),   # bench.py flags the table stale when the kernels differ
                   "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes, --kernel-trace), "
                             "eager bench steps; hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024; "
                             "hbm_bytes_per_launch averages the label's dispatches, hbm_bytes_per_step sums "
                             f"them per step ({steps} steps per pass)",
                   "kernels": res}, fh, indent=1, sort_keys=True)
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"])[:12]:
        print(f"{k:60s} {v['hbm_bytes_per_launch'] / 1e6:10.1f} MB/launch  ({v['dispatches']} dispatches)")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 2)
