"""Multi-process (gloo, world_size 2, CPU) test of the frame-shard path of
SURVEY.md §8e: every rank codes its contiguous POC block (`poc_shard`) or pair
block (`pair_shard`, bench.py's path), the decision records travel in one
collective, and rank 0's reassembled log equals the single-process run.  The per-pair compute here is the CPU oracle (this is a
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


def test_pair_shard_covers_and_balances():
    for n in (1, 2, 4, 5, 16, 30, 240):
        for world in (1, 2, 4, 8):
            blocks = [shard.pair_shard(n, world, r) for r in range(world)]
            flat = [(p, r) for b in blocks for p, refs in b for r in refs]
            assert flat == [(p, r) for p in range(1, n + 1) for r in range(min(4, p))]
            loads = [sum(len(refs) for _, refs in b) for b in blocks]
            assert max(loads) - min(loads) <= 1
            for b in blocks:  # one entry per POC, refIdx contiguous
                assert len({p for p, _ in b}) == len(b)
                assert all(refs == list(range(refs[0], refs[0] + len(refs))) for _, refs in b)
    # the c2 weak-scaling sequences (2N POCs): 2 ranks of POC 1-4 split 5 / 5
    # pairs (a whole-POC cut can do no better than 6 / 4)
    assert [sum(len(x) for _, x in shard.pair_shard(4, 2, r)) for r in range(2)] == [5, 5]
    assert shard.pair_shard(4, 2, 1) == [(3, [2]), (4, [0, 1, 2, 3])]


def test_weak_scaling_prefix_fixed_pairs_per_rank():
    """bench.py's weak scaling: the first P x N pairs of one sequence, P pairs
    on every rank (c2: P = 3, c3 / c4: P = 114)."""
    for frames in (2, 30):
        P = shard.sequence_pairs(frames)
        assert shard.frames_for_pairs(P) == frames
        for world in (1, 2, 4, 8):
            n = P * world
            F = shard.frames_for_pairs(n)
            assert shard.sequence_pairs(F) >= n > shard.sequence_pairs(F - 1)
            blocks = [shard.pair_shard(F, world, r, n) for r in range(world)]
            assert [sum(len(x) for _, x in b) for b in blocks] == [P] * world
            flat = [(p, r) for b in blocks for p, refs in b for r in refs]
            assert flat == [(p, r) for p in range(1, F + 1) for r in range(min(4, p))][:n]
    with pytest.raises(ValueError):
        shard.pair_shard(2, 1, 0, 4)


def test_merge_blocks_rejoins_split_pocs():
    blocks = [shard.pair_shard(4, 2, r) for r in range(2)]
    res = [[{(j, "FULL_2CP"): (poc, refs[j]) for j in range(len(refs))} for poc, refs in b]
           for b in blocks]
    merged = shard.merge_blocks(blocks, res)
    assert sorted(merged) == [1, 2, 3, 4]
    for poc, d in merged.items():
        assert sorted(d) == [(r, "FULL_2CP") for r in range(min(4, poc))]
        assert all(v == (poc, r) for (r, _), v in d.items())


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


def test_pack_unpack_alignment_selection():
    """Mode masks with a FULL / HALF selection (vame_pred_mask): pack writes
    only the selected PREDs and unpack expects exactly those; a result set that
    does not match the mask is refused instead of being decoded at the wrong
    offsets."""
    from vame.engine import MODE_2CP, MODE_3CP, MODE_FULL, MODE_HALF
    g = torch.Generator().manual_seed(2)
    n = {"FULL": 10, "HALF": 12}
    def rec(m):
        ncp = 3 if m.endswith("3CP") else 2
        cp = torch.randint(-2**17, 2**17, (n[m[:4]], 7), dtype=torch.int32, generator=g)
        cp[:, 0] = ncp
        if ncp == 2:
            cp[:, 5:] = 0
        return torch.randint(0, 2**31, (n[m[:4]],), dtype=torch.int64, generator=g), cp
    for modes, names in ((MODE_2CP | MODE_HALF, ("HALF_2CP",)),
                         (MODE_2CP | MODE_3CP | MODE_HALF, ("HALF_2CP", "HALF_3CP")),
                         (MODE_2CP | MODE_FULL, ("FULL_2CP",)),
                         (MODE_2CP | MODE_3CP, shard.MODES)):
        assert [k for k in shard.result_keys(1, modes)] == [(0, m) for m in names]
        res = [{(r, m): rec(m) for r in range(nr) for m in names} for nr in (2, 1)]
        lay = [(2, modes, (10, 12)), (1, modes, (10, 12))]
        flat = shard.pack(res, shard.slab_words(lay), modes=modes)
        back = shard.unpack(flat, lay)
        for a, b in zip(res, back):
            assert sorted(a) == sorted(b)
            for k in a:
                assert torch.equal(a[k][0], b[k][0]) and torch.equal(a[k][1], b[k][1])
    with pytest.raises(ValueError):
        shard.pack([{(0, "FULL_2CP"): rec("FULL_2CP"), (0, "HALF_2CP"): rec("HALF_2CP")}],
                   modes=MODE_2CP | MODE_HALF)


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
    """One rank of the GPU frame-shard run, bench.py's path (vame/seqrun.py):
    its POC block through the HIP engine (vame_affine_me_batch on cuda:0 --
    both ranks share the test box's one GPU), the compact records gathered into
    rank 0 over gloo, rank 0's sampled recompute check."""
    from vame.engine import Engine
    from vame.seqrun import ShardRun
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    eng = Engine(W, H, 0)
    run = ShardRun(eng, W, H, QP, NF, 1, world, rank, dev, seed=7)
    run.step()
    torch.cuda.synchronize()
    slabs, _ = run.gather()
    if rank == 0:
        check = run.verify(slabs)
        assert check["byte_identical"], check
        merged = shard.merge_blocks([shard.pair_shard(NF, world, r) for r in range(world)],
                                    [shard.unpack(slabs[r], run.layout(r)) for r in range(world)])
        torch.save([{f"{k[0]}:{k[1]}": (c.clone().cpu(), p.clone().cpu())
                     for k, (c, p) in merged[poc].items()} for poc in sorted(merged)],
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


class OracleEngine:
    """CPU stand-in for vame.engine.Engine with the interface ShardRun uses
    (n_cus, alloc_poc, affine_me_batch), computing with the oracle: runs the
    bench's sequence-shard path (vame/seqrun.py) on CPU ranks."""

    MODES = ("FULL_2CP", "FULL_3CP", "HALF_2CP", "HALF_3CP")

    def __init__(self, W, H):
        self.W, self.H = W, H
        self.n_ctus = O.lib().vame_oracle_num_ctus(W, H)

    def n_cus(self, align):
        return self.n_ctus * (284 if align else 201)

    def alloc_poc(self, nrefs, modes=3):
        return {(r, m): (torch.empty(self.n_cus(k >> 1), dtype=torch.int64),
                         torch.empty((self.n_cus(k >> 1), 7), dtype=torch.int32))
                for r in range(nrefs) for k, m in enumerate(self.MODES) if not ((k & 1) and not modes & 2)}

    def affine_me_batch(self, jobs, modes, extra):
        for cur, refs, lam, out in jobs:
            for r, ref in enumerate(refs):
                res = O.affine_me_pair(ref.numpy().view(np.uint16), cur.numpy().view(np.uint16), lam,
                                       extra, modes=(2, 3) if modes & 2 else (2,), nthreads=0)
                for k, m in enumerate(self.MODES):
                    if (r, m) in out:
                        c, p = res[(k >> 1, 2 + (k & 1))]
                        out[(r, m)][0].copy_(torch.from_numpy(c))
                        out[(r, m)][1].copy_(torch.from_numpy(
                            np.stack([p[f] for f in p.dtype.names], 1).astype(np.int32)))
        return [j[3] for j in jobs]


SEQ_W, SEQ_H, SEQ_N = 416, 240, 5  # 4x2 CTUs (last row 112 px high), POC 1..5 -> 11 pairs


def bench_path_worker(rank, world, port, outdir):
    """bench.py's multi-GPU path with the compute swapped for the oracle:
    ShardRun over pair_shard of one sequence, step, gather to rank 0, rank 0's
    recompute-and-compare check."""
    from vame.seqrun import ShardRun
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    run = ShardRun(OracleEngine(SEQ_W, SEQ_H), SEQ_W, SEQ_H, 27, SEQ_N, 3, world, rank,
                   torch.device("cpu"), seed=11)
    run.step()
    slabs, nbytes = run.gather()
    if rank == 0:
        check = run.verify(slabs)
        full = run.verify(slabs, full=True)
        torch.save({"slabs": slabs, "check": check, "full": full, "bytes": nbytes, "pocs": run.pocs},
                   os.path.join(outdir, "bench_path.pt"))
    else:
        assert slabs is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_bench_shard_path_two_ranks_equals_single_process(tmp_path):
    """The exact sequence-shard path bench.py --gpus N runs (vame/seqrun.py:
    one sequence, pair_shard per rank (POC 4 split between the ranks), one gather into rank 0, rank 0's sampled
    recompute check), on 2 gloo ranks: the gathered records equal a 1-rank run
    of the whole sequence word for word, and rank 0's own check passes."""
    from vame.seqrun import ShardRun
    port = free_port()
    mp.spawn(bench_path_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    got = torch.load(os.path.join(tmp_path, "bench_path.pt"), weights_only=True)
    assert got["check"]["byte_identical"] and len(got["check"]["pocs"]) >= 3
    # POC 4 is cut (rank 0: refIdx 0, rank 1: refIdx 1-3): both halves recomputed
    assert got["check"]["cut_pocs"] == [4]
    assert [4, [0], 0] in got["check"]["pocs"] and [4, [1, 2, 3], 1] in got["check"]["pocs"]
    assert got["full"]["byte_identical"] and len(got["full"]["pocs"]) == 6  # every block entry
    single = ShardRun(OracleEngine(SEQ_W, SEQ_H), SEQ_W, SEQ_H, 27, SEQ_N, 3, 1, 0,
                      torch.device("cpu"), seed=11)
    single.step()
    whole = single.slab()
    ofs = 0
    for r in range(2):
        n = shard.slab_words(shard.block_layout(shard.pair_shard(SEQ_N, 2, r), 3, single.n_cus))
        assert torch.equal(got["slabs"][r][:n], whole[ofs:ofs + n]), r
        assert not got["slabs"][r][n:].any()  # zero padding to the largest shard
        ofs += n
    assert ofs == whole.numel()
    assert got["bytes"] == 4 * got["slabs"][0].numel()


def streams_worker(rank, world, port, outdir):
    """bench.py's default weak scaling (--weak streams): every rank codes the
    same pairs of a sequence of its own; gather into rank 0 and its check."""
    from vame.seqrun import ShardRun
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    run = ShardRun(OracleEngine(SEQ_W, SEQ_H), SEQ_W, SEQ_H, 27, 2, 1, world, rank,
                   torch.device("cpu"), seed=11, n_pairs=3, streams=True)
    run.step()
    slabs, nbytes = run.gather()
    if rank == 0:
        torch.save({"slabs": slabs, "check": run.verify(slabs, full=True), "blocks": run.blocks},
                   os.path.join(outdir, "streams.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_weak_streams_two_ranks(tmp_path):
    """--weak streams on 2 gloo ranks: both ranks code POC 1-2 (3 pairs, the
    c2 shape) of their own sequence (seed_of(rank)); each gathered slab equals
    a 1-rank run with that seed, the two differ, nothing is cut, and rank 0's
    full recompute check passes."""
    from vame.seqrun import ShardRun
    port = free_port()
    mp.spawn(streams_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    got = torch.load(os.path.join(tmp_path, "streams.pt"), weights_only=True)
    assert got["blocks"] == [(1, [0]), (2, [0, 1])]
    assert got["check"]["byte_identical"] and got["check"]["cut_pocs"] == []
    assert [r for _, _, r in got["check"]["pocs"]] == [0, 0, 1, 1]
    for r in range(2):
        one = ShardRun(OracleEngine(SEQ_W, SEQ_H), SEQ_W, SEQ_H, 27, 2, 1, 2, r,
                       torch.device("cpu"), seed=11, n_pairs=3, streams=True)
        assert one.seed_of(r) == 11 + 7919 * r
        one.step()
        assert torch.equal(got["slabs"][r], one.slab()), r
    assert not torch.equal(got["slabs"][0], got["slabs"][1])


@pytest.mark.timeout(300)
def test_rank_only_block_and_verify_own():
    """A --rank-only diagnostic (bench.py / vame.distrun): rank 1's block of a
    2-rank job run alone, no process group; verify_own recomputes its first and
    last block entry and matches its own records."""
    from vame.seqrun import ShardRun
    run = ShardRun(OracleEngine(SEQ_W, SEQ_H), SEQ_W, SEQ_H, 27, SEQ_N, 3, 2, 1, torch.device("cpu"), seed=11)
    assert run.blocks == shard.pair_shard(SEQ_N, 2, 1)
    run.step()
    chk = run.verify_own()
    assert chk["byte_identical"] and [p for p, _, _ in chk["pocs"]] == [4, 5]


def test_pack_refuses_records_outside_the_compact_form():
    """The compact records drop 2-CP LB and the cost's upper half: pack refuses
    results that would not survive that (the kernels never produce them)."""
    n = 6
    cost = torch.zeros(n, dtype=torch.int64)
    cp = torch.zeros((n, 7), dtype=torch.int32)
    cp[:, 0] = 2
    shard.pack([{(0, "FULL_2CP"): (cost, cp)}])
    bad_lb = cp.clone()
    bad_lb[3, 5] = 1
    with pytest.raises(ValueError):
        shard.pack([{(0, "FULL_2CP"): (cost, bad_lb)}])
    with pytest.raises(ValueError):
        shard.pack([{(0, "FULL_2CP"): (cost + 2**31, cp)}])
    cp3 = cp.clone()
    cp3[:, 0] = 3
    cp3[:, 5:] = 7  # 3-CP records keep LB
    shard.pack([{(0, "FULL_3CP"): (cost, cp3)}])
