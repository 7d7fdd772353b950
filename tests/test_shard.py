"""Multi-process (gloo, world_size 2, CPU) test of the frame-shard path of
SURVEY.md §8e: every rank codes its contiguous POC block, the decision records
travel in one all_gather, and rank 0's reassembled log equals the
single-process run.  The per-pair compute here is the CPU oracle (this is a
test of the sharding and exchange plumbing; the GPU path is covered by
test_gpu_parity.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from vame import shard, synth
from vame.hostlogic import lambda_for_poc, ref_list

import oracle_py as O

W, H, NF, QP = 416, 240, 5, 32  # 4x2 CTUs (last row 112 px high), POC 1..5 -> 11 pairs
N_FULL, N_HALF = 8 * 201, 8 * 284


def poc_results(orig, recon, poc):
    """One POC, 2-CP only: {(refIdx, MODE): (cost, cpmv[n,7])} in engine layout."""
    res = {}
    lam = lambda_for_poc(QP, poc)
    for r, rp in enumerate(ref_list(poc)):
        out = O.affine_me_pair(recon[rp], orig[poc - 1], lam, modes=(2,), nthreads=1)
        for align, name in ((0, "FULL_2CP"), (1, "HALF_2CP")):
            c, p = out[(align, 2)]
            cp = np.stack([p[f] for f in p.dtype.names], 1).astype(np.int32)
            res[(r, name)] = (torch.from_numpy(c.copy()), torch.from_numpy(cp))
    return res


def layout(pocs):
    return [(len(ref_list(p)), 1, (N_FULL, N_HALF)) for p in pocs]


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def worker(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    orig, recon = synth.synth_sequence(W, H, NF, QP, seed=7)
    mine = shard.poc_shard(NF, world, rank)
    words = max(shard.slab_words(layout(shard.poc_shard(NF, world, r))) for r in range(world))
    slab = shard.pack([poc_results(orig, recon, p) for p in mine], words)
    slabs = shard.gather(slab, world)
    if rank == 0:
        allres = []
        for r in range(world):
            pocs = shard.poc_shard(NF, world, r)
            allres += shard.unpack(slabs[r], layout(pocs))
        torch.save([{f"{k[0]}:{k[1]}": (c.clone(), p.clone()) for k, (c, p) in res.items()}
                    for res in allres],
                   os.path.join(outdir, "gathered.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_poc_shard_covers_and_balances():
    for n in (1, 2, 5, 30, 240):
        for world in (1, 2, 4, 8):
            blocks = [shard.poc_shard(n, world, r) for r in range(world)]
            flat = [p for b in blocks for p in b]
            assert flat == list(range(1, n + 1))
            if n >= 8 * world:
                loads = [sum(shard.pairs_per_poc(p) for p in b) for b in blocks]
                assert max(loads) - min(loads) <= 4


def test_pack_unpack_roundtrip():
    g = torch.Generator().manual_seed(1)
    def rec(n, ncp):  # ABI records as the kernels write them: nCPs, 2-CP LB = 0, cost < 2^31
        cp = torch.randint(-2**17, 2**17, (n, 7), dtype=torch.int32, generator=g)
        cp[:, 0] = ncp
        if ncp == 2:
            cp[:, 5:] = 0
        return torch.randint(0, 2**31, (n,), dtype=torch.int64, generator=g), cp
    res = [{(r, m): rec(n, 3 if m.endswith("3CP") else 2)
            for r in range(nr) for m, n in (("FULL_2CP", 10), ("FULL_3CP", 10), ("HALF_2CP", 12),
                                            ("HALF_3CP", 12))}
           for nr in (1, 3)]
    lay = [(1, 3, (10, 12)), (3, 3, (10, 12))]
    flat = shard.pack(res, shard.slab_words(lay) + 5)
    back = shard.unpack(flat, lay)
    for a, b in zip(res, back):
        for k in a:
            assert torch.equal(a[k][0], b[k][0]) and torch.equal(a[k][1], b[k][1])


@pytest.mark.timeout(300)
def test_two_rank_gather_equals_single_process(tmp_path):
    port = free_port()
    mp.spawn(worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    got = torch.load(os.path.join(tmp_path, "gathered.pt"), weights_only=True)
    orig, recon = synth.synth_sequence(W, H, NF, QP, seed=7)
    assert len(got) == NF
    for poc in range(1, NF + 1):
        want = poc_results(orig, recon, poc)
        g = got[poc - 1]
        assert len(g) == len(want)
        for (r, m), (c, p) in want.items():
            gc, gp = g[f"{r}:{m}"]
            assert torch.equal(gc, c) and torch.equal(gp, p), (poc, r, m)


def gpu_worker(rank, world, port, outdir):
    """One rank of the GPU frame-shard run: its POC block through the HIP engine
    (vame_affine_me_batch on cuda:0 -- both ranks share the test box's one GPU),
    compact records all_gathered over gloo."""
    from vame.engine import Engine
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    orig, recon = synth.synth_sequence(W, H, NF, QP, seed=7)
    dev = torch.device("cuda", 0)
    eng = Engine(W, H, 0)
    mine = shard.poc_shard(NF, world, rank)
    jobs = []
    for p in mine:
        refs = [torch.from_numpy(recon[r].view(np.int16)).to(dev) for r in ref_list(p)]
        jobs.append((torch.from_numpy(orig[p - 1].view(np.int16)).to(dev), refs,
                     lambda_for_poc(QP, p), eng.alloc_poc(len(refs), 1)))
    outs = eng.affine_me_batch(jobs, 1, 0)
    torch.cuda.synchronize()
    words = max(shard.slab_words(layout(shard.poc_shard(NF, world, r))) for r in range(world))
    slabs = shard.gather(shard.pack(outs, words, dev).cpu(), world)
    if rank == 0:
        allres = []
        for r in range(world):
            allres += shard.unpack(slabs[r], layout(shard.poc_shard(NF, world, r)))
        torch.save([{f"{k[0]}:{k[1]}": (c.clone(), p.clone()) for k, (c, p) in res.items()}
                    for res in allres],
                   os.path.join(outdir, "gathered_gpu.pt"))
    dist.barrier()
    eng.close()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_two_rank_gpu_shard_equals_oracle(tmp_path):
    """The multi-GPU path with the HIP engine (2 ranks on one GPU): gathered
    decision records == the oracle's single-process results, every POC."""
    port = free_port()
    mp.spawn(gpu_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    got = torch.load(os.path.join(tmp_path, "gathered_gpu.pt"), weights_only=True)
    orig, recon = synth.synth_sequence(W, H, NF, QP, seed=7)
    assert len(got) == NF
    for poc in range(1, NF + 1):
        want = poc_results(orig, recon, poc)
        g = got[poc - 1]
        for (r, m), (c, p) in want.items():
            gc, gp = g[f"{r}:{m}"]
            assert torch.equal(gc, c) and torch.equal(gp, p), (poc, r, m)
