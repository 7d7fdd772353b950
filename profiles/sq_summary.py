#!/usr/bin/env python3
"""Per-kernel averages of the SQ counter passes written by run_sq.sh."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(float))
n = defaultdict(lambda: defaultdict(set))
for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("vame::", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[k][r["Counter_Name"]].add(r["Dispatch_Id"])
for k in sorted(acc):
    if "rocclr" in k:
        continue
    print(k)
    for c in sorted(acc[k]):
        print(f"  {c:28s} {acc[k][c] / len(n[k][c]):16.0f}")
