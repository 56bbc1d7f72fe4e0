"""Per-leg step-kernel durations from a rocprofv3 kernel trace of bench.py.

    python tools/kt_legs.py <kernel_trace.csv> [--bench bench.json] [--steps K] [--warmup W]

bench.py runs its legs in a fixed order, so the step launches of each leg are the
next dispatches of that leg's kernel instantiation in the trace:
  config 3   step_kernel<false, false, false, true, false, false> (kNt loads, N = 2^20, se_step):
             the from-reset leg's W + K launches, then the headline leg's P3 pre-roll steps
             (--preroll3, bench.py's default 1000), then the step_py
             leg's P3 + W + K
             step_kernel<false, false, false, true, false, true> (the same code, se_step_seq):
             the headline leg's W warm-up and K timed launches, then config3_literal's 10
             warm-up and 1000 timed launches
  config 4   step_kernel<false, false, true, false, false, false> (auto-reset): launches P + W .. P + W + K
             after its P pre-roll steps (--preroll4, bench.py's default 1000)
  large_n    step_kernel<false, false, false, false, false, false> (N = 2^24): the from-reset leg's
             105 launches, then the steady leg's P3 pre-roll steps and its 105 (the last)
  large_n config 4: the auto-reset kernel's last 105 launches (2^24, after its pre-roll); since
             round 5 that is the nontemporal-load instantiation (C4NT)
  config 5   policy_x3_kernel<false, false> (the fp32 policy): its first dispatches are config 5's
             W warm-up, K timed loop steps, then K policy-alone launches (bench.py run_config5);
             policy_kernel<false> (bf16): the --preroll5 pre-roll steps (eps 1.0 from reset, bench.py's
             default 300), then the bf16 leg's W + K + K in the same order. Both legs report the timed
             loop's launches; *_alone the policy-alone launches (the basis of config5's policy_ms)
For each leg this prints the average kernel duration (end - start of the dispatch, as
rocprofv3 records it) over the K timed launches, over the timed launches after the
first, the per-launch list, the idle gaps between consecutive timed launches and
(end of launch K - end of launch 1) / (K - 1), the span bench.py's events measure; with --bench, the bench line's own kernel_ms and frac
beside the figure recomputed from the trace (42 / 50 B per env-step over 8 TB/s; config 4 was 58 B
before round 5's episode-start stamps).
"""
from __future__ import annotations

import argparse
import csv
import gzip
import json

C3 = "step_kernel<false, false, false, true, false, false>"
C3S = "step_kernel<false, false, false, true, false, true>"
C4 = "step_kernel<false, false, true, false, false, false>"
C4NT = "step_kernel<false, false, true, true, false, false>"  # auto-reset with nontemporal loads (N > 2^21, round 5)
BIG = "step_kernel<false, false, false, false, false, false>"
X3 = "policy_x3_kernel<false, false>"  # se_policy_f32, config 5
PB = "policy_kernel<false>"  # se_policy (bf16)
PEAK = 8000.0


def load(path):
    rows = []
    with (gzip.open(path, "rt") if path.endswith(".gz") else open(path)) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            rows.append((s, e, name))
    rows.sort()
    return rows


def leg(rows, tag, first, count, timed, from_end=False, head=None):
    se = [(s, e) for s, e, n in rows if tag in n]
    seq = se[-count:] if from_end else se[first:first + count]
    if head is not None:
        seq = seq[:head]
    t = seq[-timed:]
    if not t:
        return None
    d = [(e - s) / 1e3 for s, e in t]
    gaps = [(t[i + 1][0] - t[i][1]) / 1e3 for i in range(len(t) - 1)]
    out = {"launches_in_trace": len(se), "timed": len(t),
           "avg_us_timed": round(sum(d) / len(d), 3),
           "avg_us_timed_after_first": round(sum(d[1:]) / max(1, len(d) - 1), 3),
           "first_timed_us": round(d[0], 3), "per_launch_us": [round(x, 3) for x in d]}
    if gaps:  # idle time between consecutive timed launches, and the events basis's span
        out["avg_gap_us"] = round(sum(gaps) / len(gaps), 3)
        out["max_gap_us"] = round(max(gaps), 3)
        out["end1_to_endK_us_per_launch"] = round((t[-1][1] - t[0][1]) / 1e3 / len(gaps), 3)
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace")
    p.add_argument("--bench")
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--n", type=int, default=1 << 20)
    p.add_argument("--preroll3", type=int, default=1000)
    p.add_argument("--preroll4", type=int, default=1000)
    p.add_argument("--preroll5", type=int, default=300)
    a = p.parse_args()
    rows = load(a.trace)
    K, W = a.steps, a.warmup
    out = {"trace": a.trace,
           "config3_from_reset": leg(rows, C3, 0, W + K, K),
           "config3": leg(rows, C3S, 0, W + K, K),
           "config3_step_py": leg(rows, C3, W + K + 2 * a.preroll3, W + K, K),
           "config4": leg(rows, C4, a.preroll4, W + K, K),
           "large_n_from_reset": leg(rows, BIG, 0, 2 * 105 + a.preroll3, 100, from_end=True, head=105),
           "large_n": leg(rows, BIG, 0, 105, 100, from_end=True),
           "config3_literal": leg(rows, C3S, W + K, 10 + 1000, 1000),
           "large_n_config4": leg(rows, C4NT, 0, 105, 100, from_end=True),
           "config5_policy_f32": leg(rows, X3, 0, W + K, K),
           "config5_policy_f32_alone": leg(rows, X3, W + K, K, K),
           "config5_policy_bf16": leg(rows, PB, a.preroll5, W + K, K),
           "config5_policy_bf16_alone": leg(rows, PB, a.preroll5 + W + K, K, K)}
    for key, b in (("config3", 42), ("config3_from_reset", 42), ("config3_step_py", 42), ("config4", 50),
                   ("config3_literal", 42)):
        if out[key]:
            us = out[key]["avg_us_timed"]
            out[key]["frac_from_trace"] = round(b * a.n / (us * 1e-6) / 1e9 / PEAK, 4)
    for key, b in (("large_n_from_reset", 42), ("large_n", 42), ("large_n_config4", 50)):
        if out[key]:
            us = out[key]["avg_us_timed"]
            out[key]["frac_from_trace"] = round(b * (1 << 24) / (us * 1e-6) / 1e9 / PEAK, 4)
    if a.bench:
        with open(a.bench) as f:
            line = next(json.loads(x) for x in f if x.startswith("{"))
        out["bench"] = {"config3": line["roofline"],
                        "config4": line.get("config4", {}).get("roofline"),
                        "config3_literal": {k: line.get("config3_literal", {}).get(k) for k in ("kernel_ms", "frac")},
                        "large_n": line.get("large_n", {}).get("roofline"),
                        "large_n_config4": line.get("large_n", {}).get("config4", {}).get("roofline")}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
