"""Medians per library of an alternating A/B record (tools/ab_*_r05.sh output, one JSON line
per run; lines naming only the library are skipped):

    python tools/ab_summary.py FILE KEY [KEY ...]
"""
import collections
import json
import statistics
import sys

f, keys = sys.argv[1], sys.argv[2:]
runs = collections.defaultdict(lambda: collections.defaultdict(list))
for line in open(f):
    r = json.loads(line)
    for k in keys:
        if k in r:
            runs[r["lib"]][k].append(r[k])
for lib, d in runs.items():
    print(lib, {k: (round(statistics.median(v), 5), v) for k, v in d.items()})
