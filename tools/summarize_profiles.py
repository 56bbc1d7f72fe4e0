"""Condense a tools/profile_round.sh output directory into profiles/<tag>/.

    python tools/summarize_profiles.py gpurun_out/prof_r01 r01

Copies the kernel_stats CSVs and writes summary.json with per-launch HBM
traffic of the step kernel from the PMC passes, corrected as MI355X_MICROARCH.md
§HBM prescribes: bytes = FETCH_SIZE(KiB) * 1024 * 2 (gfx950 reports half of a
coalesced stream's read bytes) + WRITE_SIZE(KiB) * 1024. Also refreshes
profiles/pmc_traffic.json, which bench.py reports as roofline.traffic.
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(path, kernel="step_kernel"):
    agg = defaultdict(list)
    if not os.path.exists(path):
        return {}
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def kstats(path):
    out = {}
    if not os.path.exists(path):
        return out
    for r in csv.DictReader(open(path)):
        out[r["Name"]] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                          "min_us": float(r["MinNs"]) / 1e3, "max_us": float(r["MaxNs"]) / 1e3}
    return out


def main():
    src, tag = sys.argv[1], sys.argv[2]
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    summary = {"tag": tag, "kernels": {}, "pmc": {}}
    for name in ("kt_bench", "kt_c3", "kt_c4", "kt_big", "kt_roll", "kt_pol", "kt_train"):
        f = os.path.join(src, f"{name}_kernel_stats.csv")
        if os.path.exists(f):
            shutil.copy(f, os.path.join(dst, f"{name}_kernel_stats.csv"))
            summary["kernels"][name] = kstats(f)
    b = os.path.join(src, "bench_under_rocprof.json")  # the bench's own line from the kt_bench run
    if os.path.exists(b):
        shutil.copy(b, os.path.join(dst, "bench_under_rocprof.json"))
    for name in ("fetch_c3", "write_c3", "fetch_big", "write_big", "fetch_c4", "write_c4", "fetch_c4big",
                 "write_c4big", "sq_c3", "sq2_c3"):
        summary["pmc"][name] = counters(os.path.join(src, f"pmc_{name}_counter_collection.csv"))
    n = {"c3": 1 << 20, "big": 1 << 24, "c4": 1 << 20, "c4big": 1 << 24}
    traffic = {}
    for k in ("c3", "big", "c4", "c4big"):
        fe = summary["pmc"].get(f"fetch_{k}", {}).get("FETCH_SIZE")
        wr = summary["pmc"].get(f"write_{k}", {}).get("WRITE_SIZE")
        if fe is not None and wr is not None:
            b = fe * 1024 * 2 + wr * 1024
            traffic[k] = {"bytes_per_launch": b, "bytes_per_env_step": b / n[k],
                          "fetch_kib_raw": fe, "write_kib": wr}
    summary["traffic"] = traffic
    sq = summary["pmc"].get("sq_c3", {})
    if sq.get("SQ_WAVES"):
        summary["per_wave"] = {k: v / sq["SQ_WAVES"] for k, v in sq.items() if k != "SQ_WAVES"}
    with open(os.path.join(dst, "summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    if "c3" in traffic:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w") as f:
            json.dump({"source": f"profiles/{tag}/summary.json",
                       "step_kernel_bytes_per_launch": round(traffic["c3"]["bytes_per_launch"]),
                       "workload": "config 3, N=2^20",
                       "step_kernel_auto_bytes_per_launch":
                           round(traffic["c4"]["bytes_per_launch"]) if "c4" in traffic else None,
                       "workload_auto": "config 4, N=2^20 (done-list records and the stats slab included)",
                       "step_kernel_big_bytes_per_launch":
                           round(traffic["big"]["bytes_per_launch"]) if "big" in traffic else None,
                       "workload_big": "config 3, N=2^24 (the large_n leg)",
                       "step_kernel_auto_big_bytes_per_launch":
                           round(traffic["c4big"]["bytes_per_launch"]) if "c4big" in traffic else None,
                       "workload_auto_big": "config 4, N=2^24 (the large_n config-4 leg)",
                       "correction": "FETCH_SIZE x2 (gfx950 half-count), WRITE_SIZE x1, KiB->B"},
                      f, indent=1)
    print(json.dumps({"traffic": traffic, "kernels": {k: {n: v["avg_us"] for n, v in d.items()
                                                          if "step" in n} for k, d in summary["kernels"].items()}}, indent=1))


if __name__ == "__main__":
    main()
