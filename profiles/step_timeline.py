#!/usr/bin/env python3
"""Average timeline of a bench step from a rocprofv3 kernel trace of
`bench.py --no-spans` (VAME_BENCH_KTIMING=0): the last N steps' dispatches
(one of each kernel per step, steps in order: the call's streams join at its
end), each kernel's start / end relative to the step's first dispatch.
    python profiles/step_timeline.py <kernel_trace.csv> [--last N]"""
import argparse
import csv
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--last", type=int, default=50)
a = ap.parse_args()
rows = [r for r in csv.DictReader(open(a.trace)) if "affine_me" in r["Kernel_Name"]]
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
             r["Kernel_Name"].split("(")[0].replace("void ", "").replace("vame::", "")) for r in rows)
kinds = len({n for _, _, n in iv[-80:]})
iv = iv[-kinds * a.last:]
steps = [iv[i:i + kinds] for i in range(0, len(iv) - kinds + 1, kinds)]
rel = defaultdict(lambda: [0.0, 0.0, 0])
spans = []
for st in steps:
    t0 = min(s for s, _, _ in st)
    spans.append(max(e for _, e, _ in st) - t0)
    for s, e, n in st:
        r = rel[n]
        r[0] += s - t0
        r[1] += e - t0
        r[2] += 1
print(f"{len(steps)} steps of {kinds} kernels; kernels' span per step {sum(spans) / len(spans) / 1e3:.1f} us; "
      f"step period {(iv[-1][0] - iv[0][0]) / max(len(steps) - 1, 1) / 1e3:.1f} us")
for n, (s, e, k) in sorted(rel.items(), key=lambda kv: kv[1][0]):
    print(f"  {n:28s} start {s / k / 1e3:8.1f} us  end {e / k / 1e3:8.1f} us  dur {(e - s) / k / 1e3:8.1f} us")
