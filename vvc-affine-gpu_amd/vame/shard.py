"""Frame-shard multi-GPU plumbing.

The hot path shards by frame: a (POC, ref) pair needs only orig[POC] and the
recon frame named by the deterministic reference ring (main.cpp:591-707,
replayed by `hostlogic.ref_list` on every rank), and no result feeds another
pair.  So every rank codes a contiguous block of the sequence's (POC, refIdx)
pairs (`pair_shard`; `poc_shard` is the whole-POC cut) with no collective on
the data path; the only exchange is the decision-log gather into rank 0 at the
end (one gather of equal-size padded int32 slabs, RCCL over xGMI on the GPU
box, gloo in the CPU tests).

Decision records travel compacted, as int32 words: per (POC, ref, mode) the
costs (one word each) followed by the mode's CPMV components ([n, 4] for
2 CP: LT, RT -- LB is (0, 0) and nCPs is implied; [n, 6] for 3 CP), i.e. 20 /
28 bytes per candidate CU instead of the 36 of the ABI records.  A cost always
fits int32: the SATD of a 128x128 CU is below 1024 * 2^17 < 2^28, the rate term
is a few thousand, and the initial best is MAX_LONG as the reference's OpenCL
evaluates it, 2^30.  `unpack` rebuilds the ABI records exactly.
"""
from __future__ import annotations

import torch

MODES = ("FULL_2CP", "FULL_3CP", "HALF_2CP", "HALF_3CP")


def pairs_per_poc(poc: int) -> int:
    """numRefs = min(4, POC) (main.cpp:584)."""
    return min(4, poc)


def poc_shard(n_frames: int, world: int, rank: int) -> list[int]:
    """Contiguous block of POCs 1..n_frames for `rank`, balanced by pair count
    (POC 1-3 carry fewer references).  Blocks cover every POC exactly once."""
    pocs = list(range(1, n_frames + 1))
    prefix = [0]
    for p in pocs:
        prefix.append(prefix[-1] + pairs_per_poc(p))
    total = prefix[-1]
    bounds = [0]
    for r in range(1, world):  # cut nearest to r/world of the pairs, never going back
        target = r * total / world
        i = min(range(bounds[-1], len(pocs) + 1), key=lambda j: (abs(prefix[j] - target), j))
        bounds.append(i)
    bounds.append(len(pocs))
    return pocs[bounds[rank]:bounds[rank + 1]]


def sequence_pairs(n_frames: int) -> int:
    """(POC, refIdx) pairs of a sequence of POC 1..n_frames."""
    return sum(pairs_per_poc(p) for p in range(1, n_frames + 1))


def frames_for_pairs(n_pairs: int) -> int:
    """Fewest POCs whose sequence holds at least `n_pairs` pairs."""
    f = 0
    while sequence_pairs(f) < n_pairs:
        f += 1
    return f


def pair_shard(n_frames: int, world: int, rank: int,
               n_pairs: int | None = None) -> list[tuple[int, list[int]]]:
    """Contiguous block of the sequence's (POC, refIdx) pairs for `rank`, in
    coding order (POC 1..n_frames, refIdx 0..min(4, POC)-1), as [(poc,
    [refIdx, ...]), ...].  Every pair is an independent launch in the
    reference (main.cpp:754-966, once per (POC, refIdx, PRED)), so the cut may
    fall inside a POC; the blocks hold floor / ceil of total / world pairs each,
    so no rank carries more than one pair above the mean (a POC-granular cut
    leaves up to a whole 4-ref POC of imbalance: 6 vs 4 pairs at 2 ranks of 4
    POCs).  `n_pairs` keeps only the sequence's first n_pairs pairs (weak
    scaling at a fixed pair count per rank)."""
    pairs = [(p, r) for p in range(1, n_frames + 1) for r in range(pairs_per_poc(p))]
    if n_pairs is not None:
        if n_pairs > len(pairs):
            raise ValueError("n_pairs exceeds the sequence's pairs")
        pairs = pairs[:n_pairs]
    lo, hi = rank * len(pairs) // world, (rank + 1) * len(pairs) // world
    blocks: list[tuple[int, list[int]]] = []
    for p, r in pairs[lo:hi]:
        if blocks and blocks[-1][0] == p:
            blocks[-1][1].append(r)
        else:
            blocks.append((p, [r]))
    return blocks


def block_layout(blocks, modes: int, n_cus_per_align: tuple[int, int]):
    """`unpack` / `slab_words` layout of a pair block (one entry per POC)."""
    return [(len(refs), modes, n_cus_per_align) for _, refs in blocks]


def merge_blocks(block_lists, results_lists) -> dict[int, dict]:
    """Per-POC result dicts keyed by the true refIdx, from the unpacked results
    of several ranks' pair blocks (a POC cut between two ranks is rejoined)."""
    out: dict[int, dict] = {}
    for blocks, results in zip(block_lists, results_lists):
        for (poc, refs), res in zip(blocks, results):
            d = out.setdefault(poc, {})
            for (j, mode), v in res.items():
                d[(refs[j], mode)] = v
    return out


def result_keys(nrefs: int, modes: int):
    """(refIdx, MODE) keys of one POC's results, in the fixed wire order: the
    PREDs the mode mask codes (engine.pred_mask: 2-CP / 3-CP and the
    FULL / HALF selection), refIdx outer."""
    from .engine import pred_mask
    preds = pred_mask(modes)
    return [(r, name) for r in range(nrefs) for m, name in enumerate(MODES) if (preds >> m) & 1]


def ncp_of(mode: str) -> int:
    return 3 if mode.endswith("3CP") else 2


def pack(results: list[dict], words: int | None = None, device=None, modes: int | None = None,
         validate: bool | torch.Tensor = True) -> torch.Tensor:
    """Concatenate the results of several POCs ({(ref, MODE): (cost int64[n],
    cpmv int32[n, 7])}, in POC order) into one int32 slab of compact records,
    zero padded to `words`.  With `modes`, every POC must hold exactly the
    keys `unpack` will expect for that mode mask; with `validate`, every record
    must fit the compact form (0 <= cost < 2^31, 2-CP LB = (0, 0)).  True
    checks at once (a host read, which waits for the device); a bool tensor
    instead collects the check into that flag on the device, with no wait, for
    the caller to read once after its last launch (`check_flag`)."""
    parts = []
    for res in results:
        if modes is not None:
            nrefs = max(r for r, _ in res) + 1 if res else 0
            if sorted(res, key=lambda k: (k[0], MODES.index(k[1]))) != result_keys(nrefs, modes):
                raise ValueError(f"results {sorted(res)} do not match mode mask {modes}")
        for key in sorted(res, key=lambda k: (k[0], MODES.index(k[1]))):
            cost, cpmv = res[key]
            if validate is not False:  # the compact form drops 2-CP LB and the cost's upper half
                cp7 = cpmv.reshape(-1, 7)
                over = (cost < 0).any() | (cost >= 2**31).any()
                if ncp_of(key[1]) == 2:
                    over = over | cp7[:, 5:].any()
                if isinstance(validate, torch.Tensor):
                    validate.logical_or_(over.to(validate.device))
                elif bool(over):
                    raise ValueError(f"records of {key} do not fit the compact form")
            parts.append(cost.reshape(-1).to(torch.int32))
            parts.append(cpmv.reshape(-1, 7)[:, 1:1 + 2 * ncp_of(key[1])].reshape(-1).to(torch.int32))
    flat = torch.cat(parts) if parts else torch.empty(0, dtype=torch.int32, device=device)
    if words is not None:
        if flat.numel() > words:
            raise ValueError("slab larger than the agreed size")
        flat = torch.cat([flat, flat.new_zeros(words - flat.numel())])
    return flat


def check_flag(flag: torch.Tensor) -> None:
    """Raise if a deferred `pack(..., validate=flag)` check found a record
    that does not fit the compact form (one host read)."""
    if bool(flag.item()):
        raise ValueError("decision records do not fit the compact form")


def unpack(flat: torch.Tensor, layout: list[tuple[int, int, int]]) -> list[dict]:
    """Inverse of `pack` for a list of (nrefs, modes, n_cus_per_align) POCs:
    n_cus_per_align = (FULL rows, HALF rows) of one frame."""
    out, ofs = [], 0
    for nrefs, modes, (n_full, n_half) in layout:
        res = {}
        for key in result_keys(nrefs, modes):
            n = n_half if key[1].startswith("HALF") else n_full
            ncp = ncp_of(key[1])
            cost = flat[ofs:ofs + n].to(torch.int64)
            ofs += n
            cpmv = flat.new_zeros(n, 7)
            cpmv[:, 0] = ncp
            cpmv[:, 1:1 + 2 * ncp] = flat[ofs:ofs + 2 * ncp * n].view(n, 2 * ncp)
            ofs += 2 * ncp * n
            res[key] = (cost, cpmv)
        out.append(res)
    return out


def slab_words(layout: list[tuple[int, int, int]]) -> int:
    w = 0
    for nrefs, modes, (n_full, n_half) in layout:
        for key in result_keys(nrefs, modes):
            w += (1 + 2 * ncp_of(key[1])) * (n_half if key[1].startswith("HALF") else n_full)
    return w


def poc_words(nrefs: int, modes: int, n_cus_per_align: tuple[int, int]) -> int:
    """Words of one POC's records in a slab."""
    return slab_words([(nrefs, modes, n_cus_per_align)])


def gather_to_root(slab: torch.Tensor, world: int, root: int = 0, group=None):
    """The one exchange step: every rank's equal-size slab to
    `root` (a rank of `group`, default the whole world) only (RCCL over xGMI on the GPU box: one ring-free gather into the
    root, 1/world of an all_gather's traffic).  Returns the list of slabs on
    the root, None elsewhere.  A one-rank run without a process group keeps
    its slab; with one (VAME_FORCE_PG) the slab goes through the collective."""
    import torch.distributed as dist
    if world == 1 and not (dist.is_available() and dist.is_initialized()):
        return [slab]
    rank = dist.get_rank(group)  # rank within the group; dist.gather's dst is a global rank
    dst = [torch.empty_like(slab) for _ in range(world)] if rank == root else None
    dist.gather(slab, dst, dst=root if group is None else dist.get_global_rank(group, root), group=group)
    return dst


def gather(slab: torch.Tensor, world: int, group=None) -> list[torch.Tensor]:
    """Every rank's slab to every rank (equal sizes) -- an all_gather, for
    consumers that need the whole log on every rank."""
    import torch.distributed as dist
    if world == 1:
        return [slab]
    dst = [torch.empty_like(slab) for _ in range(world)]
    dist.all_gather(dst, slab, group=group)
    return dst
