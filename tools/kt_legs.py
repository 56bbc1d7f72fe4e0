"""Per-leg step-kernel durations from a rocprofv3 kernel trace of bench.py.

    python tools/kt_legs.py <kernel_trace.csv> [--bench bench.json] [--steps K] [--warmup W]

bench.py runs its legs in a fixed order, so the step launches of each leg are the
next dispatches of that leg's kernel instantiation in the trace:
  config 3   step_kernel<false, false, false, true, false>  (kNt loads, N = 2^20): the first W + K
  config 4   step_kernel<false, false, true, false, false>  (auto-reset): launches P + W .. P + W + K
             after its P pre-roll steps (--preroll4, bench.py's default 1000)
  large_n    step_kernel<false, false, false, false, false> (N = 2^24): the last 105
For each leg this prints the average kernel duration (end - start of the dispatch, as
rocprofv3 records it) over the K timed launches, over the timed launches after the
first, and the per-launch list; with --bench, the bench line's own kernel_ms and frac
beside the figure recomputed from the trace (42 / 58 B per env-step over 8 TB/s).
"""
from __future__ import annotations

import argparse
import csv
import json

C3 = "step_kernel<false, false, false, true, false>"
C4 = "step_kernel<false, false, true, false, false>"
BIG = "step_kernel<false, false, false, false, false>"
PEAK = 8000.0


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            rows.append((s, e, name))
    rows.sort()
    return rows


def leg(rows, tag, first, count, timed, from_end=False):
    d = [(e - s) / 1e3 for s, e, n in rows if tag in n]
    seq = d[-count:] if from_end else d[first:first + count]
    t = seq[-timed:]
    if not t:
        return None
    return {"launches_in_trace": len(d), "timed": len(t),
            "avg_us_timed": round(sum(t) / len(t), 3),
            "avg_us_timed_after_first": round(sum(t[1:]) / max(1, len(t) - 1), 3),
            "first_timed_us": round(t[0], 3), "per_launch_us": [round(x, 3) for x in t]}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace")
    p.add_argument("--bench")
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--n", type=int, default=1 << 20)
    p.add_argument("--preroll4", type=int, default=1000)
    a = p.parse_args()
    rows = load(a.trace)
    K, W = a.steps, a.warmup
    out = {"trace": a.trace,
           "config3": leg(rows, C3, 0, W + K, K),
           "config4": leg(rows, C4, a.preroll4, W + K, K),
           "large_n": leg(rows, BIG, 0, 105, 100, from_end=True)}
    for key, b in (("config3", 42), ("config4", 58)):
        if out[key]:
            us = out[key]["avg_us_timed"]
            out[key]["frac_from_trace"] = round(b * a.n / (us * 1e-6) / 1e9 / PEAK, 4)
    if out["large_n"]:
        us = out["large_n"]["avg_us_timed"]
        out["large_n"]["frac_from_trace"] = round(42 * (1 << 24) / (us * 1e-6) / 1e9 / PEAK, 4)
    if a.bench:
        with open(a.bench) as f:
            line = next(json.loads(x) for x in f if x.startswith("{"))
        out["bench"] = {"config3": line["roofline"],
                        "config4": line.get("config4", {}).get("roofline"),
                        "large_n": line.get("large_n", {}).get("roofline")}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
