"""Where a bench step's time goes between kernels: from a rocprofv3 kernel
trace of `bench.py --no-spans`, the GPU's busy time (union of the two kernels'
dispatch intervals) against the span, over the last `--last` dispatch pairs
(the timed steps), and the idle gaps at step boundaries.
    python profiles/step_gaps.py <kernel_trace.csv> [--last N]"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--last", type=int, default=50)
a = ap.parse_args()
rows = [r for r in csv.DictReader(open(a.trace)) if "affine_me" in r["Kernel_Name"]]
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
iv = iv[-2 * a.last:]
busy, cur_s, cur_e = 0, None, None
gaps = []
for s, e, _ in iv:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = iv[-1][1] - iv[0][0]
quad = [e - s for s, e, n in iv if "quad" in n]
ctu = [e - s for s, e, n in iv if "ctu" in n]
print(f"{len(iv)} dispatches, span {span / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms, idle {(span - busy) / 1e6:.3f} ms "
      f"({(span - busy) / span * 100:.2f} %), {len(gaps)} gaps, mean gap {sum(gaps) / max(len(gaps), 1) / 1e3:.1f} us")
print(f"per step {span / len(quad) / 1e6:.4f} ms; quad avg {sum(quad) / len(quad) / 1e6:.4f} ms, "
      f"ctu avg {sum(ctu) / len(ctu) / 1e6:.4f} ms")
