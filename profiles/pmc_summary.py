#!/usr/bin/env python3
"""Per-kernel summary of a profile run (profiles/run_profile.sh output).

    python profiles/pmc_summary.py <prof_dir> <out.json>

Reads, under <prof_dir>:
  trace/run_kernel_stats.csv      rocprofv3 --kernel-trace --stats (durations, all dispatches)
  trace/run_kernel_trace.csv      the same run's dispatches: the timed steps' average,
  trace.log                       located with the traced run's own bench line
  pmc_fetch/, pmc_write/          one PMC pass each: FETCH_SIZE, WRITE_SIZE
  pmc_sq/                         one PMC pass: SQ_WAVES SQ_INSTS_VALU
                                  SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES ... GRBM_GUI_ACTIVE
  count.json                      profiles/count_preds.py (instrumentation build)
Every pass runs bench.py --no-spans, so each kernel's dispatches are the
step's batched launches only (no per-POC launches of other sizes mixed into the
per-launch averages).

Units and gfx950 corrections per MI355X_MICROARCH.md:
  * FETCH_SIZE / WRITE_SIZE are KiB; FETCH_SIZE counts half the bytes of wide
    coalesced reads on gfx950, so it is doubled; WRITE_SIZE is taken as is.
  * GRBM_GUI_ACTIVE is summed over the 8 XCDs: GPU cycles of a dispatch = /8.
  * SQ_ACTIVE_INST_VALU counts quad-cycles (x4 = cycles), summed over waves.
  * VALU issue ceiling: a wave64 VALU instruction issues over 2 cycles on the
    32-wide SIMD, i.e. 0.5 wave-instructions per SIMD-cycle (1024 SIMDs).
Counter passes serialize the dispatches (the two kernels do not overlap there).
"""
import csv
import json
import os
import sys
from collections import defaultdict

N_SIMD = 1024
PEAK_ISSUE = 0.5


def short(name):
    """Kernel name as the truncated trace prints it: "void vame::affine_me_quad<3>(...)"
    -> "affine_me_quad" (one kernel instance per launch mode runs per config)."""
    n = name.split("(")[0].replace("vame::", "")
    if n.startswith("void "):
        n = n[5:]
    return n.split("<")[0]


def counters(path):
    """{kernel: {counter: [value per dispatch]}} from a counter_collection.csv;
    the pseudo-counter "_duration_ns" holds each dispatch's duration."""
    per = defaultdict(lambda: defaultdict(dict))
    if not os.path.exists(path):
        return {}
    for r in csv.DictReader(open(path)):
        k, c = short(r["Kernel_Name"]), r["Counter_Name"]
        d = r["Dispatch_Id"]
        per[k][c][d] = per[k][c].get(d, 0.0) + float(r["Counter_Value"])
        if r.get("Start_Timestamp") and r.get("End_Timestamp"):
            per[k]["_duration_ns"][d] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    return {k: {c: list(v.values()) for c, v in cs.items()} for k, cs in per.items()}


def mean(v):
    return sum(v) / len(v) if v else None


def timed_dispatches(d):
    """{kernel: [duration ms of each dispatch of the traced run's timed steps]}.
    The traced run's own bench line (trace.log) gives prewarm P, warmup W,
    steps K and the kernel's launches L in the K timed steps; its dispatches,
    in order, are the P + W untimed steps' (L / K each), the timed ones, then
    any after the timed region.  Also returns that line's event averages."""
    line = None
    log = os.path.join(d, "trace.log")
    if os.path.exists(log):
        for l in open(log):
            if l.startswith("{"):
                line = json.loads(l)
    path = os.path.join(d, "trace", "run_kernel_trace.csv")
    if line is None or not os.path.exists(path):
        return {}, {}, None
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    per = defaultdict(list)
    for r in rows:
        per[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    K, W = line["steps"], line["warmup"]
    P = (line.get("prewarm") or {}).get("steps", 0)
    roof = line["roofline"]
    ts = roof.get("timed_sample") or {}
    lps = ts.get("launches_per_step")  # the quadrant kernels' launches per step (sampled events)
    dom = roof.get("kernel", "affine_me_quad")  # the line's dominant kernel
    launches = {dom: roof.get("launches")}
    events = {dom: roof.get("avg_launch_ms")}
    for k in ("affine_me_quad", "affine_me_ctu", "affine_me_half", "affine_me_ctu2", "affine_me_half2",
              "affine_me_half2w", "affine_me_half2h"):  # the others beside it
        if k != dom:
            launches[k] = roof.get(k, {}).get("launches")
            events[k] = roof.get(k, {}).get("avg_launch_ms")
    # the quadrant kernels carry events in the sampled timed steps; the
    # 128-class kernels are timed on their own steps after them
    sampled = {dom} | {k for k in launches if (roof.get(k) or {}).get("timed_on") == "the sampled timed steps"}
    out = {}
    for k, L in launches.items():
        if k in sampled and lps:  # every timed dispatch, sampled events or not
            L = lps * K
        if not L or L % K or k not in per:
            continue
        lo = (P + W) * (L // K)
        if len(per[k]) < lo + L:
            continue
        out[k] = per[k][lo:lo + L]
    return out, events, line


def main():
    d, out = sys.argv[1], sys.argv[2]
    stats = {}
    for r in csv.DictReader(open(os.path.join(d, "trace", "run_kernel_stats.csv"))):
        stats[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                                   "total_ms": float(r["TotalDurationNs"]) / 1e6,
                                   "percent": float(r["Percentage"])}
    fetch = counters(os.path.join(d, "pmc_fetch", "run_counter_collection.csv"))
    write = counters(os.path.join(d, "pmc_write", "run_counter_collection.csv"))
    sq = counters(os.path.join(d, "pmc_sq", "run_counter_collection.csv"))
    res = {"source": d, "kernels": {}}
    for k, st in stats.items():
        e = dict(st)
        f = mean(fetch.get(k, {}).get("FETCH_SIZE", []))
        w = mean(write.get(k, {}).get("WRITE_SIZE", []))
        if f is not None:
            e["fetch_size_kib_raw"] = f
            e["hbm_read_bytes_per_launch"] = 2 * f * 1024
        if w is not None:
            e["write_size_kib_raw"] = w
            e["hbm_write_bytes_per_launch"] = w * 1024
        if f is not None and w is not None:
            e["hbm_bytes_per_launch"] = e["hbm_read_bytes_per_launch"] + e["hbm_write_bytes_per_launch"]
        s = sq.get(k)
        if s and "SQ_INSTS_VALU" in s and "GRBM_GUI_ACTIVE" in s:
            sqm = {c: mean(v) for c, v in s.items()}
            gpu_cycles = sqm["GRBM_GUI_ACTIVE"] / 8.0
            if sqm.get("_duration_ns"):  # effective clock of the profiled dispatches
                e["clock_ghz"] = gpu_cycles / sqm["_duration_ns"]
            e["sq_per_launch"] = sqm
            e["sq_dispatches"] = len(s["SQ_INSTS_VALU"])
            e["valu_issue_rate"] = sqm["SQ_INSTS_VALU"] / (N_SIMD * gpu_cycles)
            e["valu_busy"] = 4.0 * sqm["SQ_ACTIVE_INST_VALU"] / (N_SIMD * gpu_cycles)
            if "SQ_WAVE_CYCLES" in sqm:
                wc = sqm["SQ_WAVE_CYCLES"]
                e["wave_cycle_split"] = {x: sqm[c] / wc for x, c in
                                         (("active_inst_any", "SQ_ACTIVE_INST_ANY"),
                                          ("wait_inst_any", "SQ_WAIT_INST_ANY"),
                                          ("wait_any", "SQ_WAIT_ANY")) if c in sqm}
        res["kernels"][k] = e
    timed, events, line = timed_dispatches(d)
    dom = ((line or {}).get("roofline") or {}).get("kernel", "affine_me_quad")
    res["dominant_kernel"] = dom
    if line is not None:  # the workload the profile was taken on (bench.py checks it against its own)
        c = line.get("config", {})
        res["profiled_workload"] = {"resolution": c.get("resolution"), "qp": c.get("qp"),
                                    "sequence_frames": c.get("sequence_frames"),
                                    "pairs_per_step_rank0": c.get("pairs_per_step_rank0"),
                                    "modes": c.get("modes"), "rank_only": c.get("rank_only"),
                                    "steps": line.get("steps"), "warmup": line.get("warmup"),
                                    "native_sha256": (line.get("native") or {}).get("sha256")}
    for k, v in timed.items():
        e = res["kernels"].setdefault(k, {})
        e["timed_dispatches"] = len(v)
        e["timed_avg_ms"] = mean(v)
        e["traced_run_event_avg_ms"] = events.get(k)
    q = res["kernels"].get(dom, {})
    res["quad_timed_avg_ms_rocprof"] = q.get("timed_avg_ms")
    res["quad_hbm_bytes_per_launch"] = q.get("hbm_bytes_per_launch")
    res["quad_avg_ms_rocprof"] = q.get("avg_ms")
    if "sq_per_launch" in q:
        # effective clock of the profiled (serialized) dispatches, GRBM cycles
        # over their own timestamps, capped at the 2.4 GHz peak (the cap if
        # the pass has no timestamps): a lower clock only understates VALU use
        res["quad_sq"] = {"insts_valu_per_launch": q["sq_per_launch"]["SQ_INSTS_VALU"],
                          "waves_per_launch": q["sq_per_launch"].get("SQ_WAVES"),
                          "valu_busy": q["valu_busy"], "issue_rate_profiled": q["valu_issue_rate"],
                          "peak_issue_rate": PEAK_ISSUE, "clock_ghz": min(q.get("clock_ghz", 2.4), 2.4),
                          "wave_cycle_split": q.get("wave_cycle_split")}
    cp = os.path.join(d, "count.json")
    if os.path.exists(cp):
        c = json.load(open(cp))
        res["executed_pred_frac"] = c["executed_pred_frac_quad"]
        res["pred_count"] = c
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
