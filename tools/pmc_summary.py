#!/usr/bin/env python3
"""Mean PMC counter value per dispatch, per kernel, from rocprofv3 --pmc CSV output (first arg: directory)."""
import csv
import glob
import sys
from collections import defaultdict

rows = []
for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    with open(f, newline="") as fh:
        rows += list(csv.DictReader(fh))
acc = defaultdict(lambda: defaultdict(list))
for r in rows:
    name = r.get("Kernel_Name", "?")[:90]
    acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} mean {sum(v) / len(v):.4g}  (n={len(v)})")
