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
ap.add_argument("--skip", type=int, default=0, help="steps to drop at the end (untimed steps after the timed ones)")
a = ap.parse_args()
rows = [r for r in csv.DictReader(open(a.trace)) if "affine_me" in r["Kernel_Name"]]
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
kinds = len({n for _, _, n in iv[-60:]})  # kernels per step (quad, ctu, half)
iv = iv[:len(iv) - kinds * a.skip] if a.skip else iv
iv = iv[-kinds * a.last:]
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
half = [e - s for s, e, n in iv if "half" in n]
print(f"{len(iv)} dispatches, span {span / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms, idle {(span - busy) / 1e6:.3f} ms "
      f"({(span - busy) / span * 100:.2f} %), {len(gaps)} gaps, mean gap {sum(gaps) / max(len(gaps), 1) / 1e3:.1f} us")
print(f"per step {span / len(quad) / 1e6:.4f} ms; quad avg {sum(quad) / len(quad) / 1e6:.4f} ms, "
      f"ctu avg {sum(ctu) / len(ctu) / 1e6:.4f} ms" +
      (f", half avg {sum(half) / len(half) / 1e6:.4f} ms" if half else ""))
# step boundaries: the gap from the end of every dispatch of step k to the first start of step k + 1
steps = [iv[i:i + kinds] for i in range(0, len(iv) - kinds + 1, kinds)]
bound = [min(s for s, _, _ in b) - max(e for _, e, _ in a_) for a_, b in zip(steps, steps[1:])]
if bound:
    bound.sort()
    print(f"step-boundary idle: median {bound[len(bound) // 2] / 1e3:.1f} us, min {bound[0] / 1e3:.1f}, "
          f"max {bound[-1] / 1e3:.1f} us over {len(bound)} boundaries")
# per step, each kernel's start / end relative to the step's first start (median over the steps)
names = sorted({n for _, _, n in iv})
rel = {n: [] for n in names}
for st in steps:
    t0 = min(s for s, _, _ in st)
    for s, e, n in st:
        rel[n].append(((s - t0) / 1e3, (e - t0) / 1e3))
print("timeline (us from the step's first start, median):")
for n in names:
    if rel[n]:
        ss = sorted(x for x, _ in rel[n])
        ee = sorted(y for _, y in rel[n])
        print(f"  {n.split('(')[0][:48]:48s} start {ss[len(ss) // 2]:8.1f}  end {ee[len(ee) // 2]:8.1f}")
