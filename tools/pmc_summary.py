"""Per-dispatch averages of rocprofv3 --pmc counters for kernels whose name contains a key.
    python tools/pmc_summary.py <counter_collection.csv> [more.csv ...] --key policy_x3
"""
import argparse
import collections
import csv
import json


def main():
    p = argparse.ArgumentParser()
    p.add_argument("csv", nargs="+")
    p.add_argument("--key", required=True)
    a = p.parse_args()
    out = {}
    for path in a.csv:
        rows = [r for r in csv.DictReader(open(path)) if a.key in r["Kernel_Name"]]
        disp = {r["Dispatch_Id"] for r in rows}
        agg = collections.defaultdict(float)
        for r in rows:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
        for k, v in agg.items():
            out[k] = v / max(len(disp), 1)
        if rows:
            out["VGPR_Count"] = int(rows[0]["VGPR_Count"])
            out["dispatches_" + path.split("/")[-1]] = len(disp)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
