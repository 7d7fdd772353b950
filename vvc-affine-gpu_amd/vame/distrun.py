"""Frame-sharded end-to-end run over N GPUs, one process per GPU (BASELINE
configs[4]): the reference's ./main contract -- CSV frames in,
the 40 per-CU decision-log CSVs out (main.cpp:293-330, :578-1003;
main_aux_functions.h:387-525) -- with the POC loop cut into contiguous
(POC, refIdx) pair blocks, one per rank (`shard.pair_shard`).

    python -m vame.distrun -f 240 -s 3840x2160 -q 32 -o orig.csv -r recon.csv \\
        -l logs/out [--gpus N] [--shard-logs [--merge-parts] | --gather-records]
        [--modes all|2cp] [--ExtraGradientIter E]

Every rank reads only the frames its block uses (`vame_read_frames_span`,
each launch's frames parsed just before they go up, beside the kernels of
the launches before), codes its block in launches of up to 32 pairs
(`vame_affine_me_batch`; the first launch small, so the GPU starts early),
and copies each launch's results to pinned host memory while the GPU runs the
next one.  The logs are written in the reference's order by one of three paths:

  default       the decision-log gather of byte counts: every rank formats
                its own block as it completes -- rank 0 into the final files,
                rank k into host memory (a deferred `vame_log_writer`) -- then
                the ranks gather their byte counts per file (one all_reduce,
                RCCL) and write their blocks into the final files at their
                offsets, all ranks in parallel (pwrite), so formatting and
                writing scale with the ranks.
  --shard-logs  per-rank files: rank 0 appends to the final files,
                rank k to its own part files `<log>.partK_*` (headerless), each
                as its launches complete, so nothing is left to write after a
                rank's last launch.  The final files are the `cat` of rank 0's
                and the parts in rank order (`vame.logs.merge_parts`, or
                `--merge-parts`: rank 0 appends them after the last rank ends).
  --gather-records  the records themselves to rank 0: every other rank packs
                its records compactly on its GPU (`shard.pack`), and after the
                last launch one gather (RCCL over xGMI) brings them to rank 0,
                which formats and writes them POC by POC (rank 0's CPU formats
                the whole log; for file systems the ranks do not share).

Blocks are contiguous in coding order, and a POC cut between two ranks is cut
at a refIdx boundary (refIdx is the outer loop of every file's rows), so both
paths give files byte-identical to a one-process run (tests/test_distrun.py).
Without a launcher, `--gpus N` starts the N ranks itself (vame.launch).
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import queue
import sys
import threading
import time

import numpy as np
import torch

from . import logs, shard
from .engine import pred_mask
from .hostlogic import lambda_for_poc, ref_list

RESOLUTIONS = ((3840, 2160), (1920, 1080), (1280, 720), (832, 480), (416, 240))  # constants.h:73-79
MAX_PAIRS = 32  # pairs per launch (vame_affine_me_batch)


def parse_args(argv=None) -> argparse.Namespace:
    """The reference's options (main.cpp:58-69) plus the frame-shard ones."""
    ap = argparse.ArgumentParser(prog="vame.distrun")
    ap.add_argument("-f", "--FramesToBeEncoded", dest="frames", type=int, required=True)
    ap.add_argument("-s", "--Resolution", dest="res", required=True)
    ap.add_argument("-q", "--QP", dest="qp", type=int, required=True)
    ap.add_argument("-o", "--OriginalFrames", dest="orig", required=True)
    ap.add_argument("-r", "--ReferenceFrames", dest="recon", required=True)
    ap.add_argument("-l", "--CpmvLogFile", dest="log", default="")
    ap.add_argument("--ExtraGradientIter", dest="extra", type=int, default=0)
    ap.add_argument("--modes", choices=("all", "2cp"), default="all")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--gather-records", action="store_true",
                    help="gather the decision records into rank 0, which formats the whole log")
    ap.add_argument("--shard-logs", action="store_true",
                    help="every rank appends its block to its own part files as it goes (<log>.partK_*)")
    ap.add_argument("--merge-parts", action="store_true",
                    help="with --shard-logs: rank 0 appends the part files to the final ones at the end")
    ap.add_argument("--rank-only", type=int, default=None, metavar="K",
                    help="run only rank K's share of a --gpus N job, alone on GPU 0 (no collective; "
                         "its logs stay part files): prices one rank of an N-GPU node on one GPU")
    a = ap.parse_args(argv)
    try:
        a.W, a.H = (int(v) for v in a.res.lower().split("x"))
    except ValueError:
        ap.error(f"bad resolution {a.res!r}")
    if (a.W, a.H) not in RESOLUTIONS:
        ap.error(f"unsupported resolution {a.W}x{a.H}")
    if a.frames < 1 or a.gpus < 1 or not 0 <= a.extra <= 64:
        ap.error("frames and gpus must be >= 1, ExtraGradientIter in 0..64")
    if a.rank_only is not None and not 0 <= a.rank_only < a.gpus:
        ap.error("--rank-only K needs 0 <= K < --gpus")
    if a.gather_records and a.shard_logs:
        ap.error("--gather-records and --shard-logs are two log paths: pick one")
    if a.merge_parts and not a.shard_logs:
        ap.error("--merge-parts goes with --shard-logs")
    a.log_path = "gather" if a.gather_records else "parts" if a.shard_logs else "place"
    if shard.sequence_pairs(a.frames) < a.gpus:  # every rank codes at least one pair
        ap.error(f"--gpus {a.gpus} needs at least as many (POC, refIdx) pairs "
                 f"({shard.sequence_pairs(a.frames)} in {a.frames} frames)")
    a.mode_mask = 3 if a.modes == "all" else 1
    return a


part_prefix = logs.part_prefix


def launch_batches(blocks, first: int = MAX_PAIRS):
    """The block's entries in launches of at most MAX_PAIRS pairs (entries
    whole); the first launches ramp up from `first` pairs, doubling (the GPU
    starts once the first launch's few frames are parsed, and each launch's
    kernels cover the parsing of the next, larger one's frames)."""
    out, cur, n = [], [], 0
    for poc, refs in blocks:
        if cur and n + len(refs) > min(MAX_PAIRS, first << len(out)):
            out.append(cur)
            cur, n = [], 0
        cur.append((poc, refs))
        n += len(refs)
    if cur:
        out.append(cur)
    return out


class _HostSlots:
    """Pinned host copies of the results of a launch, one set per slot
    (reused when the writer has finished with it)."""

    def __init__(self, n_slots: int, pin: bool):
        self.free = queue.Queue()
        self.bufs = [dict() for _ in range(n_slots)]
        self.pin = pin
        for s in range(n_slots):
            self.free.put(s)

    def host_like(self, slot: int, key, t: torch.Tensor) -> torch.Tensor:
        b = self.bufs[slot].get(key)
        if b is None or b.shape != t.shape:
            b = torch.empty(t.shape, dtype=t.dtype, pin_memory=self.pin)
            self.bufs[slot][key] = b
        return b


def run_rank(a, world: int, rank: int, engine, device, dist=None) -> dict:
    """One rank's whole run; returns its timings.  `engine` needs n_cus,
    alloc_poc and affine_me_batch (vame.engine.Engine on the GPU; the tests
    pass an oracle-backed stand-in on CPU ranks)."""
    t_start = time.perf_counter()
    W, H, modes = a.W, a.H, a.mode_mask
    n_cus = (engine.n_cus(0), engine.n_cus(1))
    cuda = device.type == "cuda"
    blocks = shard.pair_shard(a.frames, world, rank)
    T = {"rank": rank, "pairs": sum(len(r) for _, r in blocks), "pocs": len(blocks),
         "read_csv_s": 0.0, "kernel_s": 0.0, "log_write_s": 0.0, "log_bytes": 0, "gather_s": 0.0,
         "merge_s": 0.0}

    def barrier():
        if dist is not None:
            dist.barrier()

    # ---- frame ingest: only the frames this block reads (main.cpp:293-330).
    # Text lines have no fixed length, so the ranks first index the CSVs
    # together: rank r counts the newlines of chunks r, r + N, ... and one
    # all_reduce shares the counts; each rank then parses only the chunks that
    # hold its frames.
    # With the line index, each launch's frames are parsed just before they go
    # up, in the uploader thread (below), so the GPU starts after the first
    # launch's frames only and the rest of the ingest runs beside the kernels
    # (the reference reads every frame first, main.cpp:293-330); without it (a
    # one-rank run, raw frames) the block's frames are read at once, here.
    t = time.perf_counter()
    idx = {path: line_index(path, world, rank, dist, T) for path in (a.orig, a.recon)}
    T["index_s"] = time.perf_counter() - t - T.get("index_others_s", 0.0)
    d_orig, d_recon = {}, {}
    orig, recon = {}, {}  # host frames by POC
    pocs = [p for p, _ in blocks]
    need = sorted({ref_list(p)[r] for p, refs in blocks for r in refs})
    parse_s = [0.0]

    def read_into(store, path, frames):
        """Parse `frames` (POC numbers, 0-based frame index in the file) of
        `path` into `store`, one contiguous run of frames per read."""
        frames = sorted(f for f in set(frames) if f not in store)
        t0 = time.perf_counter()
        k = 0
        while k < len(frames):
            e = k
            while e + 1 < len(frames) and frames[e + 1] == frames[e] + 1:
                e += 1
            first, n = frames[k], frames[e] - frames[k] + 1
            span = None if idx[path] is None else logs.line_span(*idx[path], first * H, (first + n) * H)
            got = logs.read_frames(path, W, H, n, first=first, span=span)
            for i in range(n):
                store[first + i] = got[i]
            k = e + 1
        parse_s[0] += time.perf_counter() - t0

    overlap = blocks and idx[a.orig] is not None and idx[a.recon] is not None
    if blocks and not overlap:
        read_into(orig, a.orig, [p - 1 for p in pocs])
        read_into(recon, a.recon, need)
    T["read_csv_s"] = time.perf_counter() - t - T.get("index_others_s", 0.0)

    # frames go to the device launch by launch, ahead of the kernels, from a
    # thread and on a stream of their own (copies from pageable memory block
    # the calling thread, so the launching thread never waits for them); the
    # compute stream waits for each launch's upload event.  Results come back
    # on a third stream, overlapping the next launch.  The copy streams take an
    # explicit priority (VAME_COPY_PRIO, default -1): HIP maps streams onto 4
    # hardware queues, and a copy stream sharing the compute stream's queue
    # puts each launch's result download in front of the next launch (the
    # vame CLI measured 5.1 ms of idle GPU per 4-POC 4K launch that way).
    batches = list(launch_batches(blocks, int(os.environ.get("VAME_FIRST_LAUNCH_PAIRS", "8")) if overlap
                                  else MAX_PAIRS))
    compute = torch.cuda.current_stream(device) if cuda else None
    prio = int(os.environ.get("VAME_COPY_PRIO", "-1"))
    upstream = torch.cuda.Stream(device, priority=prio) if cuda else None
    dnstream = torch.cuda.Stream(device, priority=prio) if cuda else None
    up_ready = [threading.Event() for _ in batches]
    up_ev = [None] * len(batches)
    up_err, up_stop = [], threading.Event()

    def uploader():
        def frame(store, key, host):
            if key not in store:
                t = torch.from_numpy(np.ascontiguousarray(host).view(np.int16))
                if cuda:
                    t = t.to(device, non_blocking=True)
                    t.record_stream(compute)
                store[key] = t
        try:
            with (torch.cuda.device(device) if cuda else contextlib.nullcontext()), \
                    (torch.cuda.stream(upstream) if cuda else contextlib.nullcontext()):
                for b, batch in enumerate(batches):
                    if up_stop.is_set():
                        break
                    if overlap:  # this launch's frames, parsed now
                        read_into(orig, a.orig, [p - 1 for p, _ in batch])
                        read_into(recon, a.recon, [ref_list(p)[r] for p, refs in batch for r in refs])
                        if b == 0:
                            T["first_frames_s"] = time.perf_counter() - t_start
                    for poc, refs in batch:
                        rl = ref_list(poc)
                        frame(d_orig, poc, orig[poc - 1])
                        for r in refs:
                            frame(d_recon, rl[r], recon[rl[r]])
                    if overlap:  # host frames no later launch reads
                        last = max(p for p, _ in batch)
                        for q in [q for q in orig if q + 1 <= last]:
                            del orig[q]
                    if cuda:
                        up_ev[b] = torch.cuda.Event()
                        up_ev[b].record(upstream)
                    up_ready[b].set()
        except Exception as e:  # surfaced by the launching thread
            up_err.append(e)
        finally:
            for ev in up_ready:
                ev.set()

    up_th = threading.Thread(target=uploader, daemon=True)
    up_th.start()

    # ---- who writes what: rank 0 appends to the final files as it goes; by
    # default every other rank formats its block into host memory (a deferred
    # writer) and places it into the same files at the end; with --shard-logs
    # it appends to its own part files as it goes.  In a one-rank process group
    # (VAME_FORCE_PG) rank 0's own records take the gather path too, so the
    # collective and the writing from gathered slabs run on one GPU.
    path = a.log_path
    gather_path = bool(a.log) and path == "gather" and dist is not None
    self_gather = gather_path and world == 1
    writes_own = bool(a.log) and (rank == 0 or path != "gather") and not self_gather
    # --rank-only K (no group) and --shard-logs: rank K's rows in part files
    prefix = a.log if rank == 0 or (dist is not None and path != "parts") else part_prefix(a.log, rank)
    if a.log and (rank == 0 or dist is None or path == "parts"):
        # removeOldTraces (main.cpp:469); part files too: the deferred writer
        # places its rows at offsets without truncating, the part writer appends
        logs.remove_old(prefix)
    writer = logs.LogWriter(prefix, W, H) if (writes_own or (self_gather and rank == 0)) else None
    if writer is not None and rank > 0 and path == "place":
        writer.defer()
    slab_parts = []
    # the compact-form check of the packed records, collected on the device and
    # read once after the last launch (a per-launch read would stall the
    # launching thread until that launch finished)
    hip_pack = hasattr(engine, "pack_records")  # the HIP engine packs in one kernel
    pack_bad = torch.zeros((), dtype=torch.int32 if hip_pack else torch.bool, device=device)

    # ---- the writer thread: formats each launch's POCs once its copy landed
    slots = _HostSlots(2, cuda)
    work: queue.Queue = queue.Queue()
    err = []

    def writer_loop():
        try:
            while True:
                item = work.get()
                if item is None:
                    return
                ev, slot, batch, host = item
                if ev is not None:
                    ev.synchronize()
                t0 = time.perf_counter()
                for (poc, refs), res in zip(batch, host):
                    results = {(refs[j], name): (c.numpy(), p.numpy()) for (j, name), (c, p) in res.items()}
                    T["log_bytes"] += logs.write_poc(prefix, W, H, poc, results, writer=writer)
                T["log_write_s"] += time.perf_counter() - t0
                slots.free.put(slot)
        except Exception as e:  # surfaced after the join
            err.append(e)
            slots.free.put(-1)

    th = threading.Thread(target=writer_loop, daemon=True)
    th.start()

    # ---- the hot path: this block's launches
    spans = []
    for b, batch in enumerate(batches):
        up_ready[b].wait()
        if up_err:
            up_stop.set()
            raise up_err[0]
        jobs = []
        for poc, refs in batch:
            rl = ref_list(poc)
            jobs.append((d_orig[poc], [d_recon[rl[r]] for r in refs], lambda_for_poc(a.qp, poc),
                         engine.alloc_poc(len(refs), modes)))
        if cuda:
            compute.wait_event(up_ev[b])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        engine.affine_me_batch(jobs, modes, a.extra)
        if cuda:
            e1.record()
            spans.append((e0, e1))
        if writes_own:
            slot = slots.free.get()
            if slot < 0:
                break
            host = []
            if cuda:
                dnstream.wait_stream(torch.cuda.current_stream(device))
            with torch.cuda.stream(dnstream) if cuda else contextlib.nullcontext():
                for i, job in enumerate(jobs):
                    h = {}
                    for key, (c, p) in job[3].items():
                        hc = slots.host_like(slot, (i, key, 0), c)
                        hp = slots.host_like(slot, (i, key, 1), p)
                        hc.copy_(c, non_blocking=cuda)
                        hp.copy_(p, non_blocking=cuda)
                        if cuda:  # the launch's buffers stay allocated until the copy ran
                            c.record_stream(dnstream)
                            p.record_stream(dnstream)
                        h[key] = (hc, hp)
                    host.append(h)
                ev = None
                if cuda:
                    ev = torch.cuda.Event()
                    ev.record(dnstream)
            work.put((ev, slot, batch, host))
        elif a.log:  # gather path: compact records stay on this GPU until the gather
            if hip_pack:
                slab_parts.append(engine.pack_records([j[3] for j in jobs], modes, None, pack_bad))
            else:
                slab_parts.append(shard.pack([j[3] for j in jobs], None, device, modes=modes,
                                             validate=pack_bad))
    work.put(None)
    th.join()
    up_stop.set()
    up_th.join()
    if err:
        raise err[0]
    if overlap:  # parsed in the uploader thread, beside the launches
        T["read_csv_s"] += parse_s[0]
        T["read_csv_overlapped"] = True
    if slab_parts:
        shard.check_flag(pack_bad)
    if cuda:
        torch.cuda.synchronize()
        T["kernel_s"] = sum(x.elapsed_time(y) for x, y in spans) * 1e-3
        if spans:  # GPU idle between this rank's launches
            T["gpu_gaps_s"] = spans[0][0].elapsed_time(spans[-1][1]) * 1e-3 - T["kernel_s"]

    # ---- the decision-log gather into rank 0 (default path)
    if gather_path and (world > 1 or self_gather):
        t = time.perf_counter()
        words = max(shard.slab_words(shard.block_layout(shard.pair_shard(a.frames, world, r), modes, n_cus))
                    for r in range(world))
        mine = torch.cat(slab_parts) if slab_parts else torch.empty(0, dtype=torch.int32, device=device)
        slab = torch.cat([mine, mine.new_zeros(words - mine.numel())])
        if dist.get_backend() == "gloo":
            slab = slab.cpu()
        slabs = shard.gather_to_root(slab, world, 0)
        if cuda:
            torch.cuda.synchronize()
        T["gather_s"] = time.perf_counter() - t
        if rank == 0:
            t0 = time.perf_counter()
            for r in range(0 if self_gather else 1, world):
                o = 0
                for poc, refs in shard.pair_shard(a.frames, world, r):
                    w = shard.poc_words(len(refs), modes, n_cus)
                    res = shard.unpack(slabs[r][o:o + w], [(len(refs), modes, n_cus)])[0]
                    o += w
                    results = {(refs[j], name): (c.cpu().numpy(), p.cpu().numpy())
                               for (j, name), (c, p) in res.items()}
                    T["log_bytes"] += logs.write_poc(prefix, W, H, poc, results, writer=writer)
            T["log_write_s"] += time.perf_counter() - t0
        del slabs
    if writer is not None and rank == 0:
        writer.close()

    # ---- the default path: every rank's block into the final files at its
    # byte offsets (the sizes of the ranks before it), all ranks in parallel
    if writer is not None and rank > 0 and path == "parts":
        writer.close()  # its part files are complete
    elif writer is not None and rank > 0:
        t = time.perf_counter()
        held = writer.held_sizes()
        if dist is None:  # --rank-only K: its block alone, into its part files
            offsets = [0] * len(held)
        else:
            names = writer.files()
            sizes = torch.zeros((world, len(names)), dtype=torch.int64)
            sizes[rank] = torch.tensor(held, dtype=torch.int64)
            _all_reduce_cpu(dist, sizes)
            offsets = sizes[:rank].sum(0).tolist()
        writer.flush_at(offsets)
        writer.close()
        T["merge_s"] = time.perf_counter() - t
    elif world > 1 and a.log and path == "place" and dist is not None and rank == 0:
        names = logs.log_names(a.log)
        sizes = torch.zeros((world, len(names)), dtype=torch.int64)
        sizes[0] = torch.tensor([os.path.getsize(n) if os.path.exists(n) else 0 for n in names])
        _all_reduce_cpu(dist, sizes)
    if world > 1 and a.log and path != "gather" and dist is not None:
        barrier()  # every block is in place (or in its part files)
    if path == "parts" and a.merge_parts and rank == 0 and world > 1 and a.log:
        t = time.perf_counter()
        logs.merge_parts(a.log, world, pred_mask(modes))
        T["merge_s"] = time.perf_counter() - t
    T["overall_s"] = time.perf_counter() - t_start
    return T


def line_index(path: str, world: int, rank: int, dist, T: dict):
    """(chunk byte bounds, newline prefix counts) of a CSV, or None for raw
    frames / a one-rank run (which reads its frames from the start).  Rank r
    counts chunks r, r + world, ...; an all_reduce sums the counts.  Without
    a process group (--rank-only) the other ranks' chunks are counted here too,
    and that time is kept apart (T["index_others_s"]): on a node those chunks
    are counted by the other ranks, at the same time."""
    if world == 1 or path.endswith((".u16", ".yuv")):
        return None
    size = os.path.getsize(path)
    K = max(world, min(64 * world, size >> 22))  # chunks of >= 4 MiB
    bounds = [size * k // K for k in range(K + 1)]
    counts = torch.zeros(K, dtype=torch.int64)
    mine = list(range(rank, K, world))  # one native pass over this rank's chunks
    counts[mine] = torch.tensor(logs.count_lines_ranges(path, [(bounds[k], bounds[k + 1]) for k in mine]))
    if dist is not None:
        _all_reduce_cpu(dist, counts)
    else:
        t = time.perf_counter()
        others = [k for k in range(K) if k % world != rank]
        if others:
            counts[others] = torch.tensor(logs.count_lines_ranges(path, [(bounds[k], bounds[k + 1])
                                                                         for k in others]))
        T["index_others_s"] = T.get("index_others_s", 0.0) + time.perf_counter() - t
    prefix = [0] + torch.cumsum(counts, 0).tolist()
    return bounds, prefix


def _all_reduce_cpu(dist, t: torch.Tensor) -> None:
    """Sum a small CPU tensor over the ranks (through the GPU under RCCL)."""
    if dist.get_backend() == "nccl":
        c = t.cuda()
        dist.all_reduce(c)
        t.copy_(c.cpu())
    else:
        dist.all_reduce(t)


def report(a, per_rank: list[dict]) -> str:
    """The reference's timing block (main_aux_functions.h:1416-1446) over the
    whole job: wall-clock figures are the max over ranks, kernel time summed."""
    mx = lambda k: max(t[k] for t in per_rank)  # noqa: E731
    lines = ["=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=", "TIMING RESULTS (nanoseconds)",
             f"TOTAL_EXEC_TIME({a.frames}x),{sum(t['kernel_s'] for t in per_rank) * 1e9:f}",
             f"MAX_RANK_EXEC_TIME,{mx('kernel_s') * 1e9:f}",
             f"OVERALL({a.frames}x),{mx('overall_s'):f}",
             f"READ_CSV_TIME,{mx('read_csv_s') * 1e9:f}",
             f"LOG_WRITE_TIME,{mx('log_write_s') * 1e9:f}",
             f"LOG_GATHER_TIME,{mx('gather_s') * 1e9:f}",
             f"LOG_MERGE_TIME,{mx('merge_s') * 1e9:f}",
             f"LOG_BYTES,{sum(t['log_bytes'] for t in per_rank)}",
             "=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=",
             "DISTRUN " + json.dumps({"ranks": len(per_rank), "log_path": a.log_path,
                                      "per_rank": per_rank})]
    return "\n".join(lines)


def main(argv=None) -> int:
    a = parse_args(argv)
    from .launch import init_rank, launch_ranks
    backend = os.environ.get("VAME_DIST_BACKEND", "nccl")
    if a.rank_only is not None:  # one rank of an N-rank job, alone (no process group)
        from .engine import Engine
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        eng = Engine(a.W, a.H, 0)
        try:
            if a.log_path == "gather":  # no collective: its rows stay in its own (part) files
                a.log_path = "place"
            T = run_rank(a, a.gpus, a.rank_only, eng, dev)
        finally:
            eng.close()
        print(report(a, [T]), flush=True)
        return 0
    if "WORLD_SIZE" not in os.environ:
        if a.gpus > 1:  # no launcher: start the ranks (nothing has touched the GPU yet)
            return launch_ranks(a.gpus, ["-m", "vame.distrun"] + (sys.argv[1:] if argv is None else argv),
                                backend, "vame.distrun")
    elif int(os.environ["WORLD_SIZE"]) != a.gpus:
        print(f"vame.distrun: WORLD_SIZE={os.environ['WORLD_SIZE']} but --gpus {a.gpus}", file=sys.stderr)
        return 2
    dist, rank, dev = init_rank(a.gpus, backend)
    from .engine import Engine
    eng = Engine(a.W, a.H, dev.index)
    try:
        T = run_rank(a, a.gpus, rank, eng, dev, dist)
    finally:
        eng.close()
    per_rank = [T]
    if dist is not None:
        per_rank = [None] * a.gpus
        dist.all_gather_object(per_rank, T)
    if rank == 0:
        print(report(a, per_rank), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
