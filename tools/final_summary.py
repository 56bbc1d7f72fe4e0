"""Condense a tools/gpu_final.sh output directory into the tracked evidence files.

    python tools/final_summary.py <tag> <commit> [--dst profiles/r05/final]

Reads gpurun_out/<tag>/ (and gpurun_out/prof_<tag>/ for the PMC traffic passes) and writes
  <dst>/{bench_drv,bench_drv2,bench_under_rocprof}.json, kt_drv_kernel_stats.csv, kt_legs.json,
  size_sweep.json, smoke.log, tests_gpu.log   (copies)
  <dst>/sq_update_policy.json                  (SQ counters of the policy and update kernels,
                                                per-dispatch averages as tools/pmc_summary.py)
  <dst>/pmc/summary.json, profiles/pmc_traffic.json   (tools/summarize_profiles.py)
  profiles/rocprof_legs.json                   (the legs of kt_legs.json, what bench.py quotes)
"""
import argparse
import collections
import csv
import datetime
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NCU_SIMD = 256 * 4  # MI355X: 256 CUs x 4 SIMDs


def pmc(paths, key):
    out = {}
    for path in paths:
        if not os.path.exists(path):
            continue
        rows = [r for r in csv.DictReader(open(path)) if key in r["Kernel_Name"]]
        disp = {r["Dispatch_Id"] for r in rows}
        agg = collections.defaultdict(float)
        for r in rows:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
        for k, v in agg.items():
            out[k] = v / max(len(disp), 1)
        if rows:
            out["VGPR_Count"] = int(rows[0]["VGPR_Count"])
            out["dispatches_" + os.path.basename(path)] = len(disp)
    if out.get("SQ_WAVES"):
        w = out["SQ_WAVES"]
        out["per_wave"] = {k: round(out[k] / w, 1) for k in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS",
                                                            "SQ_INSTS_SALU") if k in out}
    if "SQ_VALU_MFMA_BUSY_CYCLES" in out:
        out["mfma_busy_cycles_per_simd"] = out["SQ_VALU_MFMA_BUSY_CYCLES"] / NCU_SIMD
    if "SQ_WAIT_ANY" in out and "SQ_WAVE_CYCLES" in out:
        out["frac_wait_any"] = round(out["SQ_WAIT_ANY"] / out["SQ_WAVE_CYCLES"], 3)
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("tag")
    p.add_argument("commit", help="the commit of the code the set was measured on")
    p.add_argument("--dst", default="profiles/r05/final")
    a = p.parse_args()
    src = os.path.join(ROOT, "gpurun_out", a.tag)
    dst = os.path.join(ROOT, a.dst)
    os.makedirs(dst, exist_ok=True)
    for f in ("bench_drv.json", "bench_drv2.json", "bench_under_rocprof.json", "kt_drv_kernel_stats.csv",
              "kt_legs.json", "size_sweep.json", "smoke.log", "tests_gpu.log"):
        if os.path.exists(os.path.join(src, f)):
            shutil.copy(os.path.join(src, f), os.path.join(dst, f))
    c = lambda n: os.path.join(src, n + "_counter_collection.csv")  # noqa: E731
    sq = {
        "policy_kernel": pmc([c("pmc_pol")], "policy_kernel<"),
        "policy_x3_kernel": pmc([c("pmc_pol32a"), c("pmc_pol32b")], "policy_x3_kernel"),
        "qtrain_tile_kernel": pmc([c("pmc_upd"), c("pmc_upd2")], "qtrain_tile_kernel"),
        "qtrain_adam_kernel": pmc([c("pmc_upd"), c("pmc_upd2")], "qtrain_adam_kernel"),
        "source": f"gpurun_out/{a.tag} pmc_pol / pmc_pol32a+b (tools/time_policy.py, 2^20 envs, bf16 / "
                  "split-bf16 f32), pmc_upd (tools/diag/update_forms.py eager) + pmc_upd2 "
                  "(tools/time_update.py, back-to-back updates): rocprofv3 --pmc passes of "
                  f"tools/gpu_final.sh {a.tag}; per-dispatch averages (tools/final_summary.py)",
    }
    with open(os.path.join(dst, "sq_update_policy.json"), "w") as f:
        json.dump(sq, f, indent=1)
    # round 6: the bf16 policy's wait counters (tools/pmc_policy_bf16.sh), the rollout kernel's
    # SQ counters and trace (tools/pmc_rollout.sh), the stepper wave's timing
    for sub, names, key in (("pmc_bf16", ("pmc_polb", "pmc_polc"), "policy_kernel<"),
                            ("rollout", ("pmc_roll_a", "pmc_roll_b"), "rollout_kernel")):
        if os.path.exists(c(names[0])):
            os.makedirs(os.path.join(dst, sub), exist_ok=True)
            with open(os.path.join(dst, sub, "summary.json"), "w") as f:
                json.dump(pmc([c(n) for n in names], key), f, indent=1)
    if os.path.exists(os.path.join(src, "kt_roll_kernel_stats.csv")):
        shutil.copy(os.path.join(src, "kt_roll_kernel_stats.csv"), os.path.join(dst, "rollout", "kt_roll_kernel_stats.csv"))
    if os.path.exists(os.path.join(src, "time_server.jsonl")):
        shutil.copy(os.path.join(src, "time_server.jsonl"), os.path.join(dst, "time_server.jsonl"))
    rel = os.path.relpath(dst, os.path.join(ROOT, "profiles"))
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "summarize_profiles.py"),
                    os.path.join(ROOT, "gpurun_out", "prof_" + a.tag), os.path.join(rel, "pmc")], check=True)
    kt = json.load(open(os.path.join(dst, "kt_legs.json")))
    legs = {"source": os.path.relpath(os.path.join(dst, "kt_legs.json"), ROOT),
            "trace": f"gpurun_out/{a.tag}/kt_drv_kernel_trace.csv (rocprofv3 --kernel-trace --stats of "
                     f"bench.py --gpus 1 --steps 20 --warmup 5, tools/gpu_final.sh {a.tag}); kernel averages "
                     f"per name in {os.path.relpath(dst, ROOT)}/kt_drv_kernel_stats.csv",
            "traced_code": f"commit {a.commit}, traced {datetime.date.today().isoformat()}"}
    for k, v in kt.items():
        if isinstance(v, dict) and "avg_us_timed" in v:
            legs[k] = {kk: vv for kk, vv in v.items() if not isinstance(vv, (list, dict))}
    with open(os.path.join(ROOT, "profiles", "rocprof_legs.json"), "w") as f:
        json.dump(legs, f, indent=1)
    print("wrote", dst, "and profiles/rocprof_legs.json, profiles/pmc_traffic.json")


if __name__ == "__main__":
    main()
