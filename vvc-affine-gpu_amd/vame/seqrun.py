"""One rank's share of a frame-sharded sequence run.

The reference codes a sequence POC by POC (main.cpp:578-585: POC 1..N, refs
from the 4-slot ring at :591-707, lambda from computeDeltaQp at :585).  No
result feeds another POC, so the POCs shard over ranks: every rank takes the
contiguous pair block `shard.pair_shard(n, world, rank)` of the SAME sequence
(same synthetic seed), synthesizes only the frames that block reads (its
originals and the recon frames of its refs), and codes it with no collective on the data
path.  The one exchange is the decision-record gather into rank 0
(`shard.gather_to_root`, RCCL over xGMI), after which rank 0 can recompute a
sample of every other rank's POCs and check the gathered records byte for byte.

With `streams` every rank instead codes the same (POC, refIdx) pairs of a
sequence of its own (seed_of(rank): the same camera motion over its own
texture): N independent streams on N GPUs, the weak-scaling form in which each
GPU's work is the 1-GPU configuration itself rather than a deeper cut of one
sequence (whose later POCs reference frames up to 23 back and converge more
slowly).

The compute engine is injected (`engine` needs `alloc_poc`, `affine_me_batch`
and `n_cus`): bench.py passes the HIP engine (vame.engine.Engine);
tests/test_shard.py passes an oracle-backed stand-in to run this exact path
under gloo on CPU ranks.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from . import shard, synth
from .hostlogic import lambda_for_poc, ref_list


class ShardRun:
    """Pair block `pair_shard(n_frames, world, rank, n_pairs)` of the sequence
    (W, H, qp, n_frames, seed) -- or with `streams` all `n_pairs` of this
    rank's own sequence -- coded with `engine` on `device`."""

    def __init__(self, engine, W: int, H: int, qp: int, n_frames: int, modes: int, world: int,
                 rank: int, device, seed: int = 0x5EED, n_pairs: int | None = None,
                 streams: bool = False):
        self.eng, self.W, self.H, self.qp, self.n = engine, W, H, qp, n_frames
        self.n_pairs = n_pairs
        self.modes, self.world, self.rank, self.device, self.seed = modes, world, rank, device, seed
        self.streams = streams
        self.n_cus = (engine.n_cus(0), engine.n_cus(1))
        self.blocks = self.blocks_of(rank)
        self.pocs = [p for p, _ in self.blocks]
        t0 = time.perf_counter()
        self.jobs = self._jobs(self.blocks)
        self.synth_s = time.perf_counter() - t0
        self.pairs = sum(len(j[1]) for j in self.jobs)
        # every rank's slab is padded to the largest shard's words (equal-size gather)
        self.words = max(shard.slab_words(self.layout(r)) for r in range(world))

    def blocks_of(self, rank: int):
        """`rank`'s (POC, [refIdx...]) block: its pair block of the one
        sequence, or with `streams` the whole `n_pairs` of its own sequence."""
        if self.streams:
            return shard.pair_shard(self.n, 1, 0, self.n_pairs)
        return shard.pair_shard(self.n, self.world, rank, self.n_pairs)

    def seed_of(self, rank: int) -> int:
        """The synthetic seed of `rank`'s frames: one sequence for all ranks,
        or with `streams` a sequence per rank (same camera motion, own texture)."""
        return self.seed + 7919 * rank if self.streams else self.seed

    def layout(self, rank: int):
        """`shard.unpack` layout of `rank`'s slab."""
        return shard.block_layout(self.blocks_of(rank), self.modes, self.n_cus)

    def _jobs(self, blocks, seed: int | None = None):
        """One engine job per (POC, [refIdx...]) entry; the job's results are
        keyed by the position in that refIdx list."""
        rps = {poc: [ref_list(poc)[i] for i in refs] for poc, refs in blocks}
        pocs = [p for p, _ in blocks]
        orig, recon = synth.synth_pocs(self.W, self.H, pocs, sorted({r for v in rps.values() for r in v}),
                                       self.qp, self.seed_of(self.rank) if seed is None else seed)
        up = lambda f: torch.from_numpy(f.view(np.int16)).to(self.device)  # noqa: E731
        d_recon = {p: up(f) for p, f in recon.items()}
        jobs = []
        for poc, refs in blocks:
            jobs.append((up(orig[poc]), [d_recon[r] for r in rps[poc]], lambda_for_poc(self.qp, poc),
                         self.eng.alloc_poc(len(refs), self.modes)))
        return jobs

    def step(self):
        """The hot path over this rank's block: one vame_affine_me_batch call."""
        if self.jobs:
            self.eng.affine_me_batch(self.jobs, self.modes, 0)

    def slab(self) -> torch.Tensor:
        """This rank's decision records packed into its compact slab: on the
        GPU in one kernel (vame_pack_records), or by shard.pack (its
        specification) for an engine without one."""
        if hasattr(self.eng, "pack_records"):
            bad = torch.zeros((), dtype=torch.int32, device=self.device)
            slab = self.eng.pack_records([j[3] for j in self.jobs], self.modes, self.words, bad)
            shard.check_flag(bad)
            return slab
        return shard.pack([j[3] for j in self.jobs], self.words, self.device, modes=self.modes)

    def exchange(self, slab: torch.Tensor):
        """The exchange step alone: every rank's packed slab into rank 0 (RCCL;
        under gloo, the CPU rehearsal of that path).  Returns (slabs on rank 0 /
        None, bytes moved into rank 0)."""
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized() and dist.get_backend() == "gloo":
            slab = slab.cpu()  # CPU rehearsal of the RCCL path
        slabs = shard.gather_to_root(slab, self.world, 0)
        return slabs, 4 * self.words * (self.world - 1)

    def gather(self):
        """The decision-record gather into rank 0 (pack + exchange): (slabs on
        rank 0 / None, bytes moved into rank 0)."""
        return self.exchange(self.slab())

    def verify_own(self) -> dict:
        """This rank's first and last block entry recomputed and compared with
        the records of its own last step (no gather: a --rank-only run)."""
        if not self.blocks:
            return {"pocs": [], "byte_identical": True}
        idx = sorted({0, len(self.blocks) - 1})
        sample = [self.blocks[i] for i in idx]
        jobs = self._jobs(sample)
        self.eng.affine_me_batch(jobs, self.modes, 0)
        ok = all(torch.equal(shard.pack([j[3]], modes=self.modes), shard.pack([self.jobs[i][3]], modes=self.modes))
                 for i, j in zip(idx, jobs))
        return {"pocs": [[p, r, self.rank] for p, r in sample], "byte_identical": ok}

    def cut_pocs(self) -> list[int]:
        """POCs whose refIdx range is split between two ranks' pair blocks."""
        if self.streams:  # every rank codes a sequence of its own
            return []
        owners: dict[int, set] = {}
        for r in range(self.world):
            for poc, _ in shard.pair_shard(self.n, self.world, r, self.n_pairs):
                owners.setdefault(poc, set()).add(r)
        return sorted(p for p, o in owners.items() if len(o) > 1)

    def verify(self, slabs, full: bool = False):
        """Rank 0: recompute block entries of every rank -- its first and last
        POC (with that rank's refs), both halves of every POC cut between two
        ranks, or with `full` every entry -- and compare their records with the
        gathered slab, word for word."""
        checked, ok = [], True
        cuts = set(self.cut_pocs())
        for r in range(self.world):
            blocks = self.blocks_of(r)
            if not blocks:
                continue
            idx = sorted(set(range(len(blocks))) if full else
                         {0, len(blocks) - 1} | {i for i, (poc, _) in enumerate(blocks) if poc in cuts})
            offs, o = [], 0
            for _, refs in blocks:
                offs.append(o)
                o += shard.poc_words(len(refs), self.modes, self.n_cus)
            for k in range(0, len(idx), 8):  # recompute in batches of 8 block entries
                part = idx[k:k + 8]
                sample = [blocks[i] for i in part]
                jobs = self._jobs(sample, self.seed_of(r))
                self.eng.affine_me_batch(jobs, self.modes, 0)
                for i, (poc, refs), job in zip(part, sample, jobs):
                    want = shard.pack([job[3]], None, self.device, modes=self.modes)
                    got = slabs[r][offs[i]:offs[i] + want.numel()]
                    ok &= bool(torch.equal(got.to(want.device), want))
                    checked.append([poc, refs, r])
        return {"pocs": checked, "cut_pocs": sorted(cuts), "byte_identical": ok}
