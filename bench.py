#!/usr/bin/env python3
"""Throughput benchmark of the affine-ME hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5]
                    [--qp QP] [--frames F] [--no-cpu-baseline] [--no-spans]

One step = the hot path over one batch of synthetic input: every (POC, refIdx)
pair of this rank's POCs (refs from the reference's 4-slot ring, lambda from
its GOP-8 model, main.cpp:578-707), FULL + HALF candidate CUs, 2-CP (and 3-CP
where the config asks for it), inputs resident in HBM, in one
vame_affine_me_batch call.  Default = BASELINE.json configs[1]: 1920x1080
QP32, 2 frames, 2-CPMV affine only (3 pairs, 196,425 candidate CUs per step).

Multi-GPU (one rank per GPU): `--gpus N` starts the N ranks
itself (fresh child processes, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set,
started before anything touches the GPU; backend nccl = RCCL over xGMI, or
VAME_DIST_BACKEND=gloo to rehearse several ranks on one GPU); under a launcher
(torchrun) that set WORLD_SIZE, WORLD_SIZE must equal --gpus.  Every rank codes the
frames of its own share, with no collective on the data path.
  c2 / c3 / c4 scale weakly: every rank codes exactly the config's (POC,
               refIdx) pairs (c2: 3, c3 / c4: 114; at N = 1 exactly the config):
               --weak streams (default): N independent sequences, one per
               rank (own synthetic texture, the same camera motion);
               --weak sequence: the first P x N pairs of ONE sequence cut into
               contiguous pair blocks shard.pair_shard(n, world, rank) (rank k
               then codes POCs up to ~3k deep, whose long-term references
               converge more slowly: a content effect, not a scaling one);
  c5           scales strongly: 240 POCs of 3840x2160 in all (configs[4]),
               contiguous pair blocks of one sequence.
After the timed steps the decision records go to rank 0 in one RCCL gather
(pack and exchange timed apart and reported as `gather`), and rank 0
recomputes the first and last POC of every rank's block and checks the
gathered records byte for byte.  Every line (N = 1 too) then carries
`frame_shard`: north star's frame shard of ONE 3840x2160 sequence
(--fs-frames, default 48 POCs = 186 pairs) over the N ranks with the gather
into rank 0 inside its timed span.  Rank 0 prints one JSON line.

`roofline`: the dominant kernel (affine_me_quad2) is VALU-issue
bound; `frac` = SQ_INSTS_VALU per launch (committed rocprofv3 profile of the
config, profiles/pmc_<config>.json) over the live launch time and the wave64
issue ceiling.  The HBM views ride beside it: measured traffic, the
algorithmic bytes of the executed predictions (`hbm_executed_frac`), and the
survey's algorithmic-byte ratio (`alg_byte_ratio`, a throughput score).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "vvc-affine-gpu_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

CONFIGS = {
    "c2": dict(W=1920, H=1080, qp=32, frames=2, modes=1, scaling="weak", steps=200, warmup=20,
               label="1920x1080 QP32, 2 frames, 2-CPMV affine only (FULL+HALF CUs)"),
    "c3": dict(W=1920, H=1080, qp=32, frames=30, modes=3, scaling="weak", steps=5, warmup=1,
               label="1920x1080 QP32, 30 frames, 2- and 3-CPMV affine (FULL+HALF CUs)"),
    "c4": dict(W=3840, H=2160, qp=32, frames=30, modes=3, scaling="weak", steps=3, warmup=1,
               label="3840x2160, 30 frames, 2- and 3-CPMV affine (FULL+HALF CUs)"),
    "c5": dict(W=3840, H=2160, qp=32, frames=240, modes=3, scaling="strong", steps=2, warmup=1,
               label="3840x2160 QP32, 240 frames frame-sharded over the GPUs, 2- and 3-CPMV "
                     "affine (FULL+HALF CUs), gather of the decision records to rank 0"),
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
N_SIMD = 1024          # 256 CUs x 4 SIMDs
# VALU issue ceiling: a wave64 VALU instruction issues over 2 cycles on a
# 32-wide SIMD (MI355X_MICROARCH.md), 0.5 wave-instructions per SIMD-cycle, at
# the 2.4 GHz peak engine clock: 1,228.8 G wave-instructions/s
VALU_PEAK_GINST = N_SIMD * 2.4 * 0.5


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--prewarm-s", type=float, default=0.25,
                    help="untimed steps until this much wall time has passed, before the warmup "
                         "steps (GPU clocks settle; 0 = none)")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--qp", type=int, default=None)
    ap.add_argument("--frames", type=int, default=None,
                    help="sequence length (c5: total POCs; c2-c4: POCs per GPU)")
    ap.add_argument("--weak", default="streams", choices=("streams", "sequence"),
                    help="weak-scaling data (c2-c4): a sequence per rank, or pair blocks of one sequence")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--rank-only", type=int, default=None, metavar="K",
                    help="diagnostic: run only rank K's block of a --gpus N job, alone on GPU 0 "
                         "(no process group, no gather): one rank of an N-GPU node, priced on one GPU")
    ap.add_argument("--no-spans", action="store_true",
                    help="skip the per-POC span step (profiling runs: identical launches only)")
    ap.add_argument("--fs-frames", type=int, default=48,
                    help="frames of the 2160p sequence the `frame_shard` record codes over the ranks "
                         "(0 = no record)")
    args = ap.parse_args()
    cfg = dict(CONFIGS[args.config])
    args.steps = cfg["steps"] if args.steps is None else args.steps
    args.warmup = cfg["warmup"] if args.warmup is None else args.warmup
    if args.qp is not None:
        cfg["qp"] = args.qp
    if args.frames is not None:
        cfg["frames"] = args.frames

    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    from vame.launch import init_rank, launch_ranks
    backend = os.environ.get("VAME_DIST_BACKEND", "nccl")
    if args.rank_only is not None:
        if not 0 <= args.rank_only < args.gpus or "WORLD_SIZE" in os.environ:
            sys.exit("bench.py: --rank-only K needs 0 <= K < --gpus and no launcher")
    elif "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:  # no launcher: start the N ranks here (nothing has touched the GPU yet)
            sys.exit(launch_ranks(args.gpus, [os.path.abspath(__file__)] + sys.argv[1:], backend,
                                  "bench.py"))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={os.environ['WORLD_SIZE']} from the launcher but --gpus {args.gpus}")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    dist, rank, dev = init_rank(world, backend)
    if args.rank_only is not None:  # shard as N ranks, run rank K's block only
        world, rank = args.gpus, args.rank_only

    from vame.engine import Engine
    from vame.metrics import pair_accounting
    from vame.seqrun import ShardRun

    W, H, qp, modes = cfg["W"], cfg["H"], cfg["qp"], cfg["modes"]
    # weak scaling: every rank codes exactly the pairs of the 1-GPU config (the
    # first frames_pairs x N pairs of one sequence, cut at pair granularity);
    # strong scaling: the config's whole sequence over the N ranks
    from vame.shard import frames_for_pairs, sequence_pairs
    weak = cfg["scaling"] == "weak"
    streams = weak and args.weak == "streams"
    n_pairs = sequence_pairs(cfg["frames"]) * (1 if streams else world) if weak else None
    n_frames = frames_for_pairs(n_pairs) if n_pairs is not None else cfg["frames"]
    ncps = (2, 3) if modes & 2 else (2,)
    eng = Engine(W, H, dev.index)
    run = ShardRun(eng, W, H, qp, n_frames, modes, world, rank, dev, n_pairs=n_pairs, streams=streams)
    log(f"[rank {rank}] POCs {run.pocs[:1]}..{run.pocs[-1:]} ({run.pairs} pairs) of {n_frames}, "
        f"frames synthesized in {run.synth_s:.1f}s")
    acc = pair_accounting(W, H, ncps)
    rows_per_step = run.pairs * acc["rows"]

    # HIP events around every per-POC launch of one extra untimed step, on the
    # stream it is issued on: the hot path's span per fused launch
    def span_step():
        ev = []
        for job in run.jobs:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            eng.affine_me_batch([job], modes, 0)
            b.record()
            ev.append((a, b))
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in ev), len(ev)

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
            torch.cuda.synchronize()

    # clocks settle before the warmup steps: a short driver run (--steps 20,
    # about 20 ms of GPU work at c2) would otherwise time a GPU still ramping up
    prewarm_steps, t_pw = 0, time.perf_counter()
    while time.perf_counter() - t_pw < args.prewarm_s:
        run.step()
        torch.cuda.synchronize()
        prewarm_steps += 1
    for _ in range(args.warmup):
        run.step()
    barrier()
    # HIP events on the quadrant kernels' dispatches of the timed steps
    # (affine_me_quad2, the dominant one, and affine_me_quad); the 128-class
    # kernels are timed on extra steps after them (timing their dispatches too
    # cost ~0.7 % of a c2 step).  Diagnostic override VAME_BENCH_KTIMING: 0 = no
    # events, 1 = every kernel in the timed steps.
    ktiming = int(os.environ.get("VAME_BENCH_KTIMING", "2"))
    # the events ride on a sample of the timed steps -- every ksample-th step
    # (VAME_BENCH_KSAMPLE, default 4) -- so the timed span carries a quarter of
    # their cost (in the engine's one-stream mode a dispatch with events costs
    # ~0.7 % of a c2 step)
    ksample = max(1, int(os.environ.get("VAME_BENCH_KSAMPLE", "4")))
    eng.set_timing(ktiming)
    # the per-step spread: HIP events around the steps that carry no kernel
    # events (i % ksample == 1; an event record is a marker packet between two
    # steps' kernels), so the spread describes a plain timed step;
    # VAME_BENCH_STEPEV=all brackets every step
    every_step = os.environ.get("VAME_BENCH_STEPEV", "sampled") == "all"
    step_ev = []
    t_start = time.perf_counter()
    for i in range(args.steps):
        sampled = i % ksample == 0
        bracket = every_step or (i % ksample == (1 if ksample > 1 else 0))
        if ksample > 1:
            eng.set_timing(ktiming if sampled else 0, keep=True)
        if bracket:
            a_, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a_.record()
        run.step()
        if bracket:
            b_.record()
            step_ev.append((a_, b_))
    barrier()
    elapsed = time.perf_counter() - t_start
    step_ms = sorted(a_.elapsed_time(b_) for a_, b_ in step_ev)
    if not step_ms:  # fewer timed steps than one sample period
        step_ms = [elapsed * 1e3 / max(args.steps, 1)]
    quad_ms, quad_n = eng.get_timing(0)    # affine_me_quad
    quad2_ms, quad2_n = eng.get_timing(6)  # affine_me_quad2
    # the 128-class kernels (128x128 CUs: affine_me_ctu2, class 3; 128x64 /
    # 64x128 CUs: affine_me_half2w / _half2h, classes 4 / 5; under PROF 1 / 2),
    # timed in the sampled timed steps with VAME_BENCH_KTIMING=1, else on extra
    # untimed steps after them
    BIG = (1, 2, 3, 4, 5)
    big_t = {k: eng.get_timing(k) for k in BIG}
    big_on = "the sampled timed steps"
    if ktiming != 1:
        big_steps = min(args.steps, 20)
        eng.set_timing(True)
        for _ in range(big_steps):
            run.step()
        big_t = {k: eng.get_timing(k) for k in BIG}
        eng.get_timing(0)
        eng.get_timing(6)
        big_on = f"{big_steps} untimed steps after the timed ones"
    eng.set_timing(False)
    span_ms, span_n = (0.0, 0) if args.no_spans else span_step()

    def all_reduce(vals, op):
        if dist is None:
            return vals
        on = dev if dist.get_backend() == "nccl" else torch.device("cpu")
        t = torch.tensor(vals, dtype=torch.float64, device=on)
        dist.all_reduce(t, op=op)
        return t.tolist()

    ops = getattr(dist, "ReduceOp", None)
    tmax = all_reduce([elapsed], ops and ops.MAX)[0]
    # whole-job totals: rows, in-frame rows, compulsory bytes (orig + ref frame + results per pair)
    rows_total, inframe_total, compulsory_total = all_reduce(
        [float(rows_per_step * args.steps), float(run.pairs * acc["rows_inframe"] * args.steps),
         float(run.pairs * (2 * W * H * 2 + acc["rows"] * 36) * args.steps)], ops and ops.SUM)
    value = rows_total / tmax

    # the one exchange step, outside the timed steps: decision records to rank 0
    # (a --rank-only diagnostic has no other ranks: it checks its own block).
    # The pack runs once untimed first (its kernels' first use), then pack and
    # exchange are timed apart, each between barriers.
    gather_rec = {"to": "rank 0", "backend": "none" if dist is None else dist.get_backend()}
    if args.rank_only is None:
        run.slab()
        barrier()
        tg = time.perf_counter()
        slab = run.slab()
        torch.cuda.synchronize()
        pack_ms = (time.perf_counter() - tg) * 1e3
        barrier()
        tg = time.perf_counter()
        slabs, gather_bytes = run.exchange(slab)
        torch.cuda.synchronize()
        exch_ms = (time.perf_counter() - tg) * 1e3
        del slab
        pack_ms, exch_ms = all_reduce([pack_ms, exch_ms], ops and ops.MAX)
        gather_rec.update({"pack_ms": pack_ms, "exchange_ms": exch_ms, "bytes_into_rank0": gather_bytes,
                           "exchange_GBps": gather_bytes / exch_ms / 1e6 if gather_bytes and exch_ms > 0
                           else None})
        gather_rec["check"] = run.verify(slabs) if rank == 0 else None
        del slabs
    else:
        gather_rec.update({"pack_ms": None, "exchange_ms": None, "bytes_into_rank0": 0,
                           "check": run.verify_own()})

    # the kernels' time per launch (sampled HIP events on their own dispatches)
    launches_per_step = -(-run.pairs // eng.max_pairs)
    prof = load_profile(args.config)
    pc = prof.get("pred_count") or {}
    # the algorithmic bytes of one launch of each kernel class (per launch:
    # the launches of a step split its pairs; the events' launches are counted)
    per_launch = lambda key: acc[key] * run.pairs / launches_per_step  # noqa: E731
    # the dominant kernel: affine_me_quad2 (the quadrant CUs of 32-128
    # sub-blocks, two per lane) when the build splits the quadrant CUs,
    # else affine_me_quad (every quadrant CU); the executed-prediction
    # fraction is counted over both quadrant kernels together
    qsplit = quad2_n > 0
    dom, dom_key = ("affine_me_quad2", "bytes_quad2") if qsplit else ("affine_me_quad", "bytes_quad")
    dom_ms, dom_n = (quad2_ms, quad2_n) if qsplit else (quad_ms, quad_n)
    quad_avg = dom_ms / dom_n if dom_n else 0.0
    roof_q = kernel_roof(quad_avg, per_launch(dom_key), prof.get("kernels", {}).get(dom),
                         pc.get("executed_pred_frac_quad"))
    # per 128-class kernel, the algorithmic bytes it carries: the 128x128 CUs
    # run in affine_me_ctu2 (the default) or in CTU items; the 128x64 / 64x128
    # CUs in affine_me_half (launches of >= 16 pairs) or in CTU items (shorter
    # launches).  A step mixing both packings leaves the CTU kernel's bytes
    # unattributed.
    ctu2 = big_t[3][1] > 0
    split = big_t[2][1] > 0 or big_t[4][1] > 0
    n_half = big_t[2][1] or big_t[4][1]
    mixed = split and (n_half != big_t[1][1] if not ctu2 else big_t[1][1] > 0)
    ctu_key = ("bytes_half" if ctu2 else "bytes_ctu") if split or ctu2 else "bytes_big"
    big_kernels = {}
    if qsplit and quad_n:  # affine_me_quad beside it: the 16-sub-block and 64x64 CUs
        big_kernels["affine_me_quad"] = {"timed_on": "the sampled timed steps", "launches": quad_n,
                                         **kernel_roof(quad_ms / quad_n, per_launch("bytes_quad1"),
                                                       prof.get("kernels", {}).get("affine_me_quad"),
                                                       pc.get("executed_pred_frac_quad"))}
    # class 4 alone: both orientations in one affine_me_half2 launch
    half2 = big_t[4][1] > 0 and big_t[5][1] == 0
    for k, name, key in ((1, "affine_me_ctu", ctu_key), (2, "affine_me_half", "bytes_half"),
                         (3, "affine_me_ctu2", "bytes_ctu"),
                         (4, "affine_me_half2", "bytes_half") if half2 else (4, "affine_me_half2w", "bytes_half_w"),
                         (5, "affine_me_half2h", "bytes_half_h")):
        ms, n = big_t[k]
        if n == 0 or (mixed and k == 1):
            continue
        big_kernels[name] = {"timed_on": big_on, "launches": n,
                             **kernel_roof(ms / n, per_launch(key), prof.get("kernels", {}).get(name),
                                           pc.get("executed_pred_frac_ctu"))}
    step_bytes = acc["bytes"] * run.pairs
    span_alg = step_bytes / (span_ms * 1e-3) / 1e9 if span_ms > 0 else 0.0
    # the whole timed step: every kernel's VALU instructions (profiled per
    # launch) and algorithmic bytes over the step's time
    step_s = elapsed / args.steps
    step_insts = None
    if roof_q.get("insts_valu_per_launch") is not None:
        step_insts = roof_q["insts_valu_per_launch"] * launches_per_step
        for name, r in big_kernels.items():
            if r.get("insts_valu_per_launch") is None:
                step_insts = None
                break
            step_insts += r["insts_valu_per_launch"] * launches_per_step
    step_alg = step_bytes / step_s / 1e9 / HBM_PEAK_GBS if step_s > 0 else 0.0

    roofline = {
        # the binding resource (rocprofv3 SQ counters, profiles/pmc_<config>.json):
        # VALU issue -- SQ_INSTS_VALU per launch over this run's launch time,
        # against the wave64 issue ceiling of 1,024 SIMDs at the peak clock
        "bound": "valu",
        "kernel": dom,
        # the engine issues affine_me_quad2 on a side stream and the 128-class
        # kernels and affine_me_quad on the caller's stream (VAME_STREAMS=2,
        # DESIGN §4): they run side by side, so this kernel's launch time
        # includes their share of the GPU; step.valu_frac counts every kernel's
        # instructions over the step
        "concurrent_with": sorted(big_kernels) if os.environ.get("VAME_STREAMS", "2") != "1" else [],
        "achieved": roof_q.get("valu_Ginst_per_s"),
        "peak": VALU_PEAK_GINST,
        "unit": "G VALU wave-instructions/s",
        "frac": roof_q.get("valu_frac"),
        # SQ_ACTIVE_INST_VALU: the VALU pipe's busy cycles (most of the kernel's
        # instructions hold it for more than the 2 issue cycles)
        "busy": roof_q.get("valu_busy"),
        # measured HBM bytes per launch (PMC FETCH_SIZE x 2 + WRITE_SIZE)
        "traffic": roof_q.get("hbm_bytes_per_launch"),
        "hbm_measured_frac": roof_q.get("hbm_measured_frac"),
        # the prescribed HBM view: the algorithmic window bytes of
        # the predictions the exact early exit runs, over the launch time and
        # 8 TB/s; and the same for every algorithmic prediction -- a throughput
        # score (it exceeds 1 once the early exit skips enough), not a fraction
        "hbm_executed_frac": roof_q.get("hbm_executed_frac"),
        "alg_byte_ratio": roof_q.get("alg_byte_ratio"),
        "executed_pred_frac": pc.get("executed_pred_frac_quad"),
        "avg_launch_ms": quad_avg,
        "launches": quad_n,
        # the timed steps whose quadrant dispatches carry the events
        "timed_sample": {"every": ksample, "steps": len(range(0, args.steps, ksample)) if ktiming else 0,
                         "launches_per_step": launches_per_step},
        "alg_bytes_per_launch": roof_q["alg_bytes_per_launch"],
        "insts_valu_per_launch": roof_q.get("insts_valu_per_launch"),
        "wave_cycle_split": roof_q.get("wave_cycle_split"),
        # the same kernel's average under rocprofv3 over the timed dispatches
        # of a traced run of this config, the committed profile the counter
        # fields come from, the workload it was taken on, whether that is this
        # line's workload and whether it ran the library this line loaded
        "rocprof_avg_ms": (prof.get("kernels", {}).get(dom) or {}).get("timed_avg_ms"),
        "profile": prof.get("profile"),
        "profiled_workload": prof.get("profiled_workload"),
        "profile_matches_workload": profile_matches(prof, cfg, run, world, args.rank_only),
        "profile_same_library": profile_same_library(prof),
        **big_kernels,
        # every kernel of the timed step together
        "step": {"valu_frac": (step_insts / step_s / 1e9 / VALU_PEAK_GINST) if step_insts and step_s > 0
                 else None,
                 "hbm_executed_frac": step_alg * pc["executed_pred_frac"] if pc.get("executed_pred_frac")
                 else None,
                 "alg_byte_ratio": step_alg},
        "fused_poc_launch": {"alg_byte_ratio": span_alg / HBM_PEAK_GBS,
                             "avg_launch_ms": span_ms / max(span_n, 1),
                             "alg_bytes_per_launch": step_bytes / max(span_n, 1)},
    }

    result = {
        "metric": "candidate CU-blocks/s at 1080p QP32; bit-exact CPMV/cost match vs reference",
        "value": value,
        "unit": "CU-blocks/s",
        "n_gpus": 1 if args.rank_only is not None else world,
        "steps": args.steps,
        "warmup": args.warmup,
        "prewarm": {"seconds": args.prewarm_s, "steps": prewarm_steps},
        "ms_per_step": tmax * 1e3 / args.steps,
        # rank 0's per-step GPU times (HIP events around the timed steps that
        # carry no kernel-timing events)
        "step_ms": {"median": step_ms[len(step_ms) // 2], "min": step_ms[0], "max": step_ms[-1],
                    "steps": len(step_ms)},
        "world": {"size": world, "backend": "none" if dist is None else dist.get_backend(),
                  "launcher": os.environ.get("VAME_LAUNCHER", "external" if world > 1 else "none"),
                  # VAME_FORCE_PG=1: a one-rank process group, so the N-GPU
                  # collectives (init, all_reduce, gather) run on one GPU
                  "forced_pg": args.rank_only is None and world == 1 and dist is not None},
        "higher_is_better": True,
        "scaling": cfg["scaling"],
        # which multi-GPU form this line measures: weak scaling over
        # independent sequences ("streams", the default) or over pair blocks
        # of one sequence ("sequence"); c5 is the north star's frame shard of
        # one 240-frame sequence (strong scaling); every line also carries the
        # frame shard of one 2160p sequence (`frame_shard`)
        "scaling_form": ("streams" if streams else "sequence") if weak else "frame-shard",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic",
        "config": {"workload": cfg["label"], "resolution": f"{W}x{H}", "qp": qp,
                   "sequence_frames": n_frames, "sequence_pairs": n_pairs or sequence_pairs(n_frames),
                   "pocs_rank0": len(run.pocs),
                   "pairs_per_step_rank0": run.pairs, "rows_per_step_rank0": rows_per_step,
                   "rows_per_step_all": rows_total / args.steps,
                   "modes": "2cp+3cp" if modes & 2 else "2cp",
                   "parallelism": (f"frame-shard x{world} (a sequence of its own per rank)" if streams else
                                   f"frame-shard x{world} (pair_shard of one sequence)"),
                   "scaling_form_note": ("N independent sequences (each rank codes the 1-GPU config "
                                         "on its own synthetic sequence); the frame shard of one "
                                         "sequence is `frame_shard` (and --config c5)" if streams else
                                         "the first P x N pairs of one sequence in contiguous pair "
                                         "blocks (deeper POCs on higher ranks)" if weak else
                                         "240 POCs of one sequence in contiguous pair blocks over "
                                         "the ranks"),
                   **({"rank_only": {"rank": rank, "of": world}} if args.rank_only is not None else {})},
        "roofline": roofline,
        # SURVEY §8(d) companions: in-frame candidates (the rows the kernels
        # predict; out-of-frame rows are logged with their initial cost) and the
        # compulsory bytes (orig + ref frame + results per pair) over the step
        "value_inframe": inframe_total / tmax,
        "compulsory": {"bytes_per_step_all": compulsory_total / args.steps,
                       "GBps": compulsory_total / tmax / 1e9 if tmax > 0 else 0.0},
        "gather": gather_rec,
    }
    result["native"] = native_record()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"], result["parity_sample"] = cpu_baseline(run, acc, ncps, W, H, modes)
    eng.close()
    del run
    torch.cuda.empty_cache()
    # north star's frame shard of one sequence, with the RCCL gather of the
    # decision records into rank 0 inside its timed span (every N, N = 1 too;
    # a c5 line is that shard itself, over the whole 240 frames)
    if args.fs_frames > 0 and args.rank_only is None and args.config != "c5":
        result["frame_shard"] = frame_shard_record(args.fs_frames, dist, rank, world, dev, barrier,
                                                   all_reduce, ops)
    if dist is not None:
        dist.barrier()
    if rank == 0 or args.rank_only is not None:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def native_record() -> dict:
    """The HIP library this run loaded, tied to the build that made it
    (__graft_entry__.build() writes lib/build_record.json)."""
    import hashlib
    from vame import _lib
    rec = {"lib": os.path.relpath(_lib.LIB_PATH, REPO),
           "sha256": hashlib.sha256(open(_lib.LIB_PATH, "rb").read()).hexdigest()}
    path = os.path.join(os.path.dirname(_lib.LIB_PATH), "build_record.json")
    if os.path.exists(path):
        b = json.load(open(path))
        built = b.get("artefacts", {}).get("vvc-affine-gpu_amd/lib/libvame.so", {})
        rec["build"] = {"git_head": b.get("git_head"), "mode": b.get("mode"),
                        "matches_loaded_lib": built.get("sha256") == rec["sha256"]}
    return rec


def profile_matches(prof: dict, cfg: dict, run, world: int, rank_only) -> bool | None:
    """Whether the committed profile was taken on this line's workload (same
    resolution, QP, modes, pairs per step and rank block), so that its
    rocprof average and counters describe the launches this line times."""
    pw = prof.get("profiled_workload")
    if not pw:
        return None
    ro = {"rank": rank_only, "of": world} if rank_only is not None else None
    return (pw.get("resolution") == f"{cfg['W']}x{cfg['H']}" and pw.get("qp") == cfg["qp"]
            and pw.get("modes") == ("2cp+3cp" if cfg["modes"] & 2 else "2cp")
            and pw.get("pairs_per_step_rank0") == run.pairs and pw.get("rank_only") == ro)


def profile_same_library(prof: dict) -> bool | None:
    """Whether the committed profile's run loaded the same HIP library (its
    sha256) as this line: its kernel times describe this build's kernels."""
    pw = prof.get("profiled_workload") or {}
    if not pw.get("native_sha256"):
        return None
    return pw["native_sha256"] == native_record()["sha256"]


def load_profile(config: str) -> dict:
    """The committed counter profile of this config (profiles/pmc_<config>.json,
    written by profiles/pmc_summary.py from rocprofv3 passes over identical
    launches): per kernel its rocprof timed average, HBM bytes per launch
    (FETCH_SIZE x 2 + WRITE_SIZE), SQ counters per launch (SQ_INSTS_VALU, ...)
    and VALU busy fraction; the executed-prediction count of the
    instrumentation build; the workload and library it was taken with."""
    path = os.path.join(REPO, "profiles", f"pmc_{config}.json")
    if not os.path.exists(path):
        return {}
    p = json.load(open(path))
    return {"kernels": p.get("kernels", {}), "pred_count": p.get("pred_count"),
            "profiled_workload": p.get("profiled_workload"), "profile": os.path.relpath(path, REPO)}


def kernel_roof(avg_ms: float, alg_bytes: float, prof_kernel: dict | None, exec_frac: float | None) -> dict:
    """One kernel's roofline figures from its live launch time and its
    committed profile:
      valu_frac          SQ_INSTS_VALU per launch / (avg launch time x the wave64
                         issue ceiling of 1,024 SIMDs at the 2.4 GHz peak clock:
                         0.5 wave-instructions per SIMD-cycle) -- the bound
      valu_busy          SQ_ACTIVE_INST_VALU x 4 / (1,024 SIMD x GPU cycles), profiled
      hbm_measured_frac  measured HBM bytes per launch / time / 8 TB/s
      hbm_executed_frac  algorithmic bytes x executed-prediction fraction / time / 8 TB/s
      alg_byte_ratio     algorithmic bytes / time / 8 TB/s (a throughput score:
                         it charges predictions the exact early exit skips)"""
    pk = prof_kernel or {}
    out = {"avg_launch_ms": avg_ms, "alg_bytes_per_launch": alg_bytes}
    if avg_ms <= 0:
        return out
    alg = alg_bytes / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
    out["alg_byte_ratio"] = alg
    out["hbm_executed_frac"] = alg * exec_frac if exec_frac else None
    hbm = pk.get("hbm_bytes_per_launch")
    out["hbm_bytes_per_launch"] = hbm
    out["hbm_measured_frac"] = hbm / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if hbm else None
    insts = (pk.get("sq_per_launch") or {}).get("SQ_INSTS_VALU")
    if insts:
        g = insts / (avg_ms * 1e-3) / 1e9
        out.update({"insts_valu_per_launch": insts, "valu_Ginst_per_s": g, "valu_frac": g / VALU_PEAK_GINST,
                    "valu_busy": pk.get("valu_busy"), "wave_cycle_split": pk.get("wave_cycle_split"),
                    "rocprof_avg_ms": pk.get("timed_avg_ms")})
    return out


def frame_shard_record(n_frames: int, dist, rank: int, world: int, dev, barrier, all_reduce, ops) -> dict:
    """North star's multi-GPU form at every N: ONE synthetic 3840x2160 QP32
    sequence of `n_frames` POCs (2- and 3-CP, FULL + HALF) cut into contiguous
    (POC, refIdx) pair blocks over the ranks (shard.pair_shard), coded with no
    collective on the data path, and the decision records packed and gathered
    into rank 0 (RCCL over xGMI) INSIDE the timed span: barrier, then kernels +
    pack + gather; the span is the max over ranks.  One untimed warm-up pass
    first (the kernels' first use, clocks).  The gather then runs once more
    between barriers, timing the exchange alone.  Rank 0 recomputes the first
    and last block entry of every rank and both halves of every cut POC and
    compares the gathered records word for word."""
    from vame.engine import Engine
    from vame.metrics import pair_accounting
    from vame.seqrun import ShardRun
    from vame.shard import sequence_pairs
    Wf, Hf, qp, modes = 3840, 2160, 32, 3
    t_syn = time.perf_counter()
    eng = Engine(Wf, Hf, dev.index)
    run = ShardRun(eng, Wf, Hf, qp, n_frames, modes, world, rank, dev)
    syn_s = time.perf_counter() - t_syn
    acc = pair_accounting(Wf, Hf, (2, 3))
    run.step()  # untimed warm-up
    run.slab()
    barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    run.step()
    e1.record()
    slab = run.slab()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    slabs, nbytes = run.exchange(slab)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    kern_ms = e0.elapsed_time(e1)
    del slabs
    # the exchange alone, between barriers
    barrier()
    t3 = time.perf_counter()
    slabs, _ = run.exchange(slab)
    torch.cuda.synchronize()
    exch_ms = (time.perf_counter() - t3) * 1e3
    del slab
    span_ms, kmax, kernels_pack_ms, gather_ms, exch_ms = all_reduce(
        [(t2 - t0) * 1e3, kern_ms, (t1 - t0) * 1e3, (t2 - t1) * 1e3, exch_ms], ops and ops.MAX)
    kmin = all_reduce([kern_ms], ops and ops.MIN)[0]
    check = run.verify(slabs) if rank == 0 else None
    del slabs
    total_pairs = sequence_pairs(n_frames)
    rows = total_pairs * acc["rows"]
    rec = {"workload": f"{Wf}x{Hf} QP{qp}, {n_frames} frames ({total_pairs} (POC, refIdx) pairs), "
                       f"2- and 3-CPMV affine (FULL+HALF CUs), contiguous pair blocks of one sequence over "
                       f"{world} rank(s), decision records gathered into rank 0",
           "frames": n_frames, "pairs": total_pairs, "pairs_rank0": run.pairs, "rows": rows,
           "ms": span_ms, "rows_per_s": rows / (span_ms * 1e-3) if span_ms > 0 else None,
           "kernel_ms": {"max": kmax, "min": kmin},
           "kernels_pack_ms_max": kernels_pack_ms, "gather_ms_max": gather_ms,
           "exchange_ms": exch_ms, "bytes_into_rank0": nbytes,
           "exchange_GBps": nbytes / exch_ms / 1e6 if nbytes and exch_ms > 0 else None,
           "backend": "none" if dist is None else dist.get_backend(),
           "synth_s_rank0": syn_s, "check": check}
    eng.close()
    del run
    torch.cuda.empty_cache()
    return rec


def host_cpus():
    """(threads the CPU baseline uses, description).  The baseline uses every
    core this process may run on (sched affinity), capped by the cgroup CPU
    quota and by OMP_NUM_THREADS where the host sets one (the GPU box gives
    each GPU a 16-CPU share and sets OMP_NUM_THREADS=16)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    omp = int(omp) if omp and omp.isdigit() and int(omp) > 0 else None
    threads = min(x for x in (aff, quota, omp) if x)
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return threads, {"cpu_model": model, "host_cpus": os.cpu_count(), "affinity_cpus": aff,
                     "cgroup_quota_cpus": quota, "omp_num_threads": omp}


def cpu_baseline(run, acc, ncps, W, H, modes, min_seconds=10.0):
    """The CPU oracle (C restatement, OpenMP) on a bounded sample of the same
    workload: the step's (POC, refIdx) pairs in order, cycling until at least
    `min_seconds` of CPU work -- and a bit-exact check of the GPU output of
    every pair it ran against it."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_py as O
    from vame import synth
    from vame.hostlogic import ref_list
    threads, cpus = host_cpus()
    orig, recon = synth.synth_pocs(W, H, run.pocs, sorted({p for q in run.pocs for p in ref_list(q)}),
                                   run.qp, run.seed)
    # (POC, refIdx, ref POC, lambda, the job's results, key position in the job)
    pairs = [(poc, r, ref_list(poc)[r], job[2], job[3], j) for (poc, refs), job in zip(run.blocks, run.jobs)
             for j, r in enumerate(refs)]
    names = (("FULL_2CP", (0, 2)), ("FULL_3CP", (0, 3)), ("HALF_2CP", (1, 2)), ("HALF_3CP", (1, 3)))
    rows, dt, ok, checked, k = 0, 0.0, True, set(), 0
    while dt < min_seconds or k == 0:
        poc, r, rp, lam, out, j = pairs[k % len(pairs)]
        t0 = time.perf_counter()
        res = O.affine_me_pair(recon[rp], orig[poc], lam, 0, modes=ncps, nthreads=threads)
        dt += time.perf_counter() - t0
        rows += acc["rows"]
        if (poc, r) not in checked:
            checked.add((poc, r))
            for name, key in names:
                if key not in res:
                    continue
                c, p = out[(j, name)]
                oc, op = res[key]
                gp = p.cpu().numpy()[:, 1:]
                opp = np.stack([op[f] for f in ("LTx", "LTy", "RTx", "RTy", "LBx", "LBy")], 1)
                ok &= bool((c.cpu().numpy() == oc).all() and (gp == opp).all())
        k += 1
    base = {"value": rows / dt, "unit": "CU-blocks/s", "cores": threads, "kind": "port",
            "sample": f"{W}x{H}, {k} (POC, refIdx) pairs of the step's {len(pairs)} in order "
                      f"(cycled), FULL+HALF {'+'.join(f'{n}CP' for n in ncps)}, {rows} candidate "
                      f"CUs, oracle/vame_oracle.c OpenMP x{threads}, {dt:.1f}s",
            **cpus}
    return base, {"pairs": len(checked), "rows": len(checked) * acc["rows"], "bit_exact": ok}


if __name__ == "__main__":
    main()
