#!/usr/bin/env python3
"""Forecast of the driver's multi-GPU bench curve (`bench.py --gpus N`, N = 2,
4, 8), committed before the driver measures it.  Every
rank's share is coded here, one rank after another, on ONE MI355X:

  * `frame_shard` (north star's form: one 3840x2160 QP32 sequence of 48 POCs,
    186 (POC, refIdx) pairs, 2+3 CP, cut into contiguous pair blocks by
    shard.pair_shard): per rank its pairs, kernel time (one
    vame_affine_me_batch call, median of 3 after a warm-up), pack time
    (vame_pack_records) and slab bytes;
  * the weak `streams` line (c2: every rank codes the 1-GPU config, 3 pairs of
    1080p 2-CP, on a sequence of its own): per rank the step time.

The forecast of a span is the maximum over ranks of (kernels + pack) plus the
gather of the other ranks' padded slabs into rank 0, priced at an assumed
RCCL ingress rate (the only exchange; no rank waits for another before it).
gpurun only:  python3 profiles/scale_forecast.py > profiles/r06_scale_forecast.txt
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vvc-affine-gpu_amd"))

import torch  # noqa: E402

from vame.engine import Engine  # noqa: E402
from vame.metrics import pair_accounting  # noqa: E402
from vame.seqrun import ShardRun  # noqa: E402
from vame.shard import sequence_pairs  # noqa: E402

# assumed RCCL gather ingress into rank 0 over xGMI (7 links x ~153 GB/s peak
# per direction; a gather's senders each use their own link): low / high
INGRESS_GBPS = (300.0, 700.0)


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2]


def main():
    dev = torch.device("cuda", 0)
    out = {"frame_shard": {}, "weak_streams_c2": {}, "assumed_ingress_GBps": INGRESS_GBPS}
    # ---- frame_shard: 48 frames of 2160p, 2+3 CP
    Wf, Hf, nf = 3840, 2160, 48
    rows = sequence_pairs(nf) * pair_accounting(Wf, Hf, (2, 3))["rows"]
    torch.cuda.init()
    free0 = torch.cuda.mem_get_info(0)[0]
    eng = Engine(Wf, Hf, 0)
    out["context_bytes_2160p"] = free0 - torch.cuda.mem_get_info(0)[0]  # scratch + templates, 32 pairs
    print(f"2160p context (vame_create, 32 pairs per launch): {out['context_bytes_2160p'] / 2**20:.0f} MiB",
          flush=True)
    for N in (1, 2, 4, 8):
        ranks = []
        for k in range(N):
            run = ShardRun(eng, Wf, Hf, 32, nf, 3, N, k, dev)
            kern = timed(run.step)
            pack = timed(run.slab)
            ranks.append({"rank": k, "pairs": run.pairs, "pocs": [run.pocs[0], run.pocs[-1]],
                          "kernel_ms": round(kern, 3), "pack_ms": round(pack, 3),
                          "slab_bytes": run.words * 4})
            print(f"frame_shard N={N} rank {k}: {run.pairs} pairs POC {run.pocs[0]}..{run.pocs[-1]} "
                  f"kernels {kern:.2f} ms pack {pack:.2f} ms", flush=True)
            del run
            torch.cuda.empty_cache()
        compute = max(r["kernel_ms"] + r["pack_ms"] for r in ranks)
        into0 = (N - 1) * ranks[0]["slab_bytes"]
        gather = [into0 / (g * 1e6) for g in INGRESS_GBPS]
        span = [compute + g for g in reversed(gather)]  # (low, high) ms
        out["frame_shard"][N] = {
            "ranks": ranks, "max_kernels_plus_pack_ms": round(compute, 3),
            "bytes_into_rank0": into0, "gather_ms": [round(g, 2) for g in reversed(gather)],
            "forecast_ms": [round(s, 2) for s in span],
            "forecast_rows_per_s": [round(rows / (s * 1e-3)) for s in reversed(span)]}
    eng.close()
    # ---- weak streams, c2: 1080p QP32, 2 frames, 2-CP, a sequence per rank
    free0 = torch.cuda.mem_get_info(0)[0]
    eng = Engine(1920, 1080, 0)
    out["context_bytes_1080p"] = free0 - torch.cuda.mem_get_info(0)[0]
    print(f"1080p context: {out['context_bytes_1080p'] / 2**20:.0f} MiB", flush=True)
    for N in (1, 2, 4, 8):
        per = []
        for k in range(N):
            run = ShardRun(eng, 1920, 1080, 32, 2, 1, N, k, dev, n_pairs=3, streams=True)

            def steps(run=run):
                for _ in range(50):
                    run.step()
            per.append(round(timed(steps) / 50, 4))
            del run
        out["weak_streams_c2"][N] = {"per_rank_ms": per, "max_ms": max(per),
                                     "forecast_efficiency_vs_rank0": round(per[0] / max(per), 4)}
        print(f"weak c2 N={N}: per-rank ms/step {per}", flush=True)
    eng.close()
    print(json.dumps(out))


if __name__ == "__main__":
    t = time.time()
    main()
    print(f"scale_forecast {time.time() - t:.1f} s", flush=True)
