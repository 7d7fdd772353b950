#!/usr/bin/env python3
"""Probe: the c2 step (one vame_affine_me_batch call) launched eagerly vs
replayed from a HIP graph captured with torch.cuda.graph.  Prints ms/step for
both and checks the replayed results equal the eager ones.  gpurun only."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vvc-affine-gpu_amd"))

import torch  # noqa: E402

from vame import synth  # noqa: E402
from vame.engine import Engine  # noqa: E402
from vame.hostlogic import lambda_for_poc, ref_list  # noqa: E402


def main():
    W, H, nf, qp, modes, steps = 1920, 1080, 2, 32, 1, 50
    orig, recon = synth.synth_sequence(W, H, nf, qp)
    dev = torch.device("cuda", 0)
    d_o = [torch.from_numpy(orig[k].view("int16")).to(dev) for k in range(nf)]
    d_r = [torch.from_numpy(recon[k].view("int16")).to(dev) for k in range(nf)]
    eng = Engine(W, H, 0)
    jobs = [(d_o[p - 1], [d_r[r] for r in ref_list(p)], lambda_for_poc(qp, p),
             eng.alloc_poc(len(ref_list(p)), modes)) for p in range(1, nf + 1)]

    def step():
        eng.affine_me_batch(jobs, modes, 0)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    ref = {k: (v[0].clone(), v[1].clone()) for k, v in jobs[1][3].items()}
    t = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t) / steps * 1e3

    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        step()
    for k in ref:
        jobs[1][3][k][0].zero_()
    g.replay()
    torch.cuda.synchronize()
    ok = all(torch.equal(jobs[1][3][k][0], ref[k][0]) and torch.equal(jobs[1][3][k][1], ref[k][1])
             for k in ref)
    t = time.perf_counter()
    for _ in range(steps):
        g.replay()
    torch.cuda.synchronize()
    graph = (time.perf_counter() - t) / steps * 1e3
    print(f"eager {eager:.4f} ms/step, graph {graph:.4f} ms/step, graph results equal: {ok}")


if __name__ == "__main__":
    main()
