"""Per-wave averages of SQ counters for the step kernel from tools/profile_sq.sh output."""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
agg = defaultdict(list)
for f in glob.glob(f"{d}/*_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "step_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
avg = {k: sum(v) / len(v) for k, v in agg.items()}
w = avg.get("SQ_WAVES", 1.0)
for k in sorted(avg):
    print(f"{k:28s} total {avg[k]:14.0f}   per wave {avg[k] / w:10.1f}")
