"""The frame-sharded end-to-end path (vame/distrun.py; VERDICT r2
item 2): CSV frames in, the 40 decision logs out, over several ranks -- both
log paths (the gather into rank 0, and --shard-logs with the parallel part
merge) give files byte-identical to the reference's writer (restated in
tests/oracle_log.py from main_aux_functions.h:387-525) applied to one
process's results, including a POC cut between two ranks.

CPU tests run the exact rank code under gloo with the HIP engine swapped for
the CPU oracle (results precomputed once and looked up by frame content); the
GPU tests run `python -m vame.distrun --gpus 2` (two ranks sharing the test
box's GPU, gloo) against the single-process `vame` CLI."""
import hashlib
import os
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from vame import distrun, logs, shard
from vame.hostlogic import lambda_for_poc, ref_list
from vame.synth import synth_sequence, write_csv

import oracle_log as OL
import oracle_py as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODES = ("FULL_2CP", "FULL_3CP", "HALF_2CP", "HALF_3CP")
KEYS = {(0, 2): 0, (0, 3): 1, (1, 2): 2, (1, 3): 3}


def digest(a: np.ndarray) -> str:
    return hashlib.sha1(np.ascontiguousarray(a).view(np.uint8)).hexdigest()


def oracle_results(orig, recon, qp, modes=(2, 3)):
    """{(cur digest, ref digest, lambda): {(align, ncp): (cost, cpmv[n, 7])}} for
    every pair of the sequence, plus the same keyed by (POC, refIdx)."""
    by_frames, by_pair = {}, {}
    for poc in range(1, orig.shape[0] + 1):
        lam = lambda_for_poc(qp, poc)
        for r, rp in enumerate(ref_list(poc)):
            res = O.affine_me_pair(recon[rp], orig[poc - 1], lam, modes=modes, nthreads=0)
            res = {k: (torch.from_numpy(c.copy()),
                       torch.from_numpy(np.stack([p[f] for f in p.dtype.names], 1).astype(np.int32)))
                   for k, (c, p) in res.items()}
            by_frames[(digest(orig[poc - 1]), digest(recon[rp]), np.float32(lam).item())] = res
            by_pair[(poc, r)] = res
    return by_frames, by_pair


def expected_logs(prefix, W, H, n, by_pair):
    """The restated reference writer over the sequence, in the host's order."""
    for poc in range(1, n + 1):
        for r in range(min(4, poc)):
            res = by_pair[(poc, r)]
            for key, pred in sorted(KEYS.items(), key=lambda kv: kv[1]):
                if key not in res:
                    continue
                if poc == 1 and r == 0:
                    OL.write_headers(prefix, pred)
                OL.append(prefix, pred, W, H, poc, r, *(t.numpy() for t in res[key]))


class LookupEngine:
    """CPU stand-in for vame.engine.Engine (n_cus, alloc_poc, affine_me_batch)
    serving precomputed oracle results by frame content."""

    def __init__(self, W, H, table):
        self.n_ctus = O.lib().vame_oracle_num_ctus(W, H)
        self.table = table

    def n_cus(self, align):
        return self.n_ctus * (284 if align else 201)

    def alloc_poc(self, nrefs, modes=3):
        return {(r, m): (torch.empty(self.n_cus(k >> 1), dtype=torch.int64),
                         torch.empty((self.n_cus(k >> 1), 7), dtype=torch.int32))
                for r in range(nrefs) for k, m in enumerate(MODES) if not ((k & 1) and not modes & 2)}

    def affine_me_batch(self, jobs, modes, extra):
        assert extra == 0
        for cur, refs, lam, out in jobs:
            for r, ref in enumerate(refs):
                res = self.table[(digest(cur.numpy().view(np.uint16)), digest(ref.numpy().view(np.uint16)),
                                  np.float32(lam).item())]
                for (r2, m), (c, p) in out.items():
                    if r2 == r:
                        k = MODES.index(m)
                        c.copy_(res[(k >> 1, 2 + (k & 1))][0])
                        p.copy_(res[(k >> 1, 2 + (k & 1))][1])
        return [j[3] for j in jobs]


def rank_worker(rank, world, port, argv, table_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a = distrun.parse_args(argv)
    table = torch.load(table_path, weights_only=True)
    distrun.run_rank(a, world, rank, LookupEngine(a.W, a.H, table), torch.device("cpu"), dist)
    dist.barrier()
    dist.destroy_process_group()


def compare_dirs(a, b):
    fa, fb = sorted(os.listdir(a)), sorted(os.listdir(b))
    assert fa == fb
    for f in fa:
        assert (a / f).read_bytes() == (b / f).read_bytes(), f
    return fa


SEQ = dict(W=416, H=240, n=6, qp=27, seed=21)  # POC 1..6: 18 pairs


@pytest.fixture(scope="module")
def seq(tmp_path_factory):
    tmp = tmp_path_factory.mktemp("dist")
    orig, recon = synth_sequence(SEQ["W"], SEQ["H"], SEQ["n"], SEQ["qp"], seed=SEQ["seed"])
    write_csv(str(tmp / "orig.csv"), orig)
    write_csv(str(tmp / "recon.csv"), recon)
    by_frames, by_pair = oracle_results(orig, recon, SEQ["qp"])
    torch.save(by_frames, tmp / "table.pt")
    exp = tmp / "expected"
    exp.mkdir()
    expected_logs(str(exp / "log"), SEQ["W"], SEQ["H"], SEQ["n"], by_pair)
    return tmp


def run_ranks(tmp, world, name, extra=()):
    out = tmp / name
    out.mkdir()
    argv = ["-f", str(SEQ["n"]), "-s", f"{SEQ['W']}x{SEQ['H']}", "-q", str(SEQ["qp"]),
            "-o", str(tmp / "orig.csv"), "-r", str(tmp / "recon.csv"), "-l", str(out / "log"), *extra]
    if world == 1:
        a = distrun.parse_args(argv)
        table = torch.load(tmp / "table.pt", weights_only=True)
        distrun.run_rank(a, 1, 0, LookupEngine(a.W, a.H, table), torch.device("cpu"))
    else:
        from vame.launch import free_port
        mp.spawn(rank_worker, args=(world, free_port(), argv, str(tmp / "table.pt")), nprocs=world,
                 join=True)
    return out


def test_launch_batches_and_cuts():
    blocks = shard.pair_shard(240, 8, 1)
    batches = distrun.launch_batches(blocks)
    assert [e for b in batches for e in b] == blocks
    assert all(sum(len(r) for _, r in b) <= distrun.MAX_PAIRS for b in batches)
    # a small first launch (the GPU starts once its frames are parsed), doubling up to full ones
    small = distrun.launch_batches(blocks, 8)
    assert [e for b in small for e in b] == blocks
    sizes = [sum(len(r) for _, r in b) for b in small]
    assert sizes[0] <= 8 and sizes[1] <= 16 and sizes[2] <= 32 and sizes[1] > 8
    assert all(s <= distrun.MAX_PAIRS for s in sizes) and max(sizes) > 16
    # the 6-POC sequence over 2 / 3 ranks cuts POC 4 / POC 5 between ranks
    for world, cut in ((2, [4]), (3, [5])):
        owners = {}
        for r in range(world):
            for p, _ in shard.pair_shard(6, world, r):
                owners.setdefault(p, []).append(r)
        assert [p for p, o in owners.items() if len(o) > 1] == cut


@pytest.mark.timeout(600)
def test_one_rank_logs_byte_identical(seq):
    assert len(compare_dirs(run_ranks(seq, 1, "one"), seq / "expected")) == 40


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 3])
def test_gathered_logs_byte_identical(seq, world):
    """--gather-records: records gathered into rank 0, which writes every POC."""
    assert len(compare_dirs(run_ranks(seq, world, f"gather{world}", ["--gather-records"]), seq / "expected")) == 40


def self_gather_worker(rank, world, port, argv, table_path):
    rank_worker(rank, world, port, argv, table_path)


@pytest.mark.timeout(600)
def test_one_rank_group_gathers_its_own_records(seq):
    """A one-rank process group (what VAME_FORCE_PG=1 forms): rank 0's records
    take the gather path -- packed per launch with the deferred device-side
    check, gathered through the collective, unpacked and written from the
    slab -- and the 40 files equal the reference writer's."""
    out = seq / "selfgather"
    out.mkdir()
    argv = ["-f", str(SEQ["n"]), "-s", f"{SEQ['W']}x{SEQ['H']}", "-q", str(SEQ["qp"]),
            "-o", str(seq / "orig.csv"), "-r", str(seq / "recon.csv"), "-l", str(out / "log"),
            "--gather-records"]
    from vame.launch import free_port
    mp.spawn(self_gather_worker, args=(1, free_port(), argv, str(seq / "table.pt")), nprocs=1, join=True)
    assert len(compare_dirs(out, seq / "expected")) == 40


def test_pack_deferred_check():
    """shard.pack with a device flag collects the compact-form check without a
    host read; check_flag raises once a record does not fit."""
    n = 5
    good = {(0, "FULL_2CP"): (torch.arange(n, dtype=torch.int64), torch.zeros((n, 7), dtype=torch.int32))}
    flag = torch.zeros((), dtype=torch.bool)
    shard.pack([good], validate=flag, modes=None)
    shard.check_flag(flag)
    bad_cost = {(0, "FULL_2CP"): (torch.full((n,), 2**31, dtype=torch.int64), torch.zeros((n, 7), dtype=torch.int32))}
    cp = torch.zeros((n, 7), dtype=torch.int32)
    cp[2, 6] = 4  # a 2-CP record with LB != 0
    bad_lb = {(0, "HALF_2CP"): (torch.zeros(n, dtype=torch.int64), cp)}
    for bad in (bad_cost, bad_lb):
        f = torch.zeros((), dtype=torch.bool)
        shard.pack([good, bad], validate=f)
        with pytest.raises(ValueError):
            shard.check_flag(f)
        with pytest.raises(ValueError):
            shard.pack([bad])


def test_rank_only_part_files_are_replaced(seq):
    """--rank-only K (K > 0) writes its block into <log>.partK_* at offset 0
    without truncating: stale longer part files from an earlier run must be
    removed first."""
    out = seq / "rankonly"
    out.mkdir()
    argv = ["-f", str(SEQ["n"]), "-s", f"{SEQ['W']}x{SEQ['H']}", "-q", str(SEQ["qp"]),
            "-o", str(seq / "orig.csv"), "-r", str(seq / "recon.csv"), "-l", str(out / "log"),
            "--gpus", "2", "--rank-only", "1"]
    a = distrun.parse_args(argv)
    table = torch.load(seq / "table.pt", weights_only=True)
    pre = distrun.part_prefix(a.log, 1)
    names = [os.path.basename(n) for n in __import__("vame.logs", fromlist=["x"]).log_names(pre)]
    for n in names:  # stale, longer than any real part
        (out / n).write_bytes(b"X" * 10_000_000)
    distrun.run_rank(a, 2, 1, LookupEngine(a.W, a.H, table), torch.device("cpu"))
    first = {n: (out / n).read_bytes() for n in names if (out / n).exists()}
    assert first and all(b"X" * 64 not in v for v in first.values())
    distrun.run_rank(a, 2, 1, LookupEngine(a.W, a.H, table), torch.device("cpu"))
    assert {n: (out / n).read_bytes() for n in names if (out / n).exists()} == first


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 3])
def test_placed_logs_byte_identical(seq, world):
    """The default path: every rank writes its block, placed at its offsets in
    the final files; no part file is left behind."""
    out = run_ranks(seq, world, f"place{world}")
    assert len(compare_dirs(out, seq / "expected")) == 40


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 3])
def test_shard_logs_cat_merge_byte_identical(seq, world):
    """--shard-logs: rank 0 writes the final files, rank k its
    headerless part files, each as it goes; the `cat` of the parts in rank
    order (logs.merge_parts) is the one-process logs byte for byte."""
    out = run_ranks(seq, world, f"shard{world}", ["--shard-logs"])
    files = sorted(os.listdir(out))
    assert len(files) == 40 * world and sum(".part" in f for f in files) == 40 * (world - 1)
    # the same bytes as a plain cat of rank 0's file and the parts
    name = logs.log_names(str(out / "log"))[0]
    cat = b"".join(open(n, "rb").read() for n in [name] + [logs.log_names(logs.part_prefix(str(out / "log"), r))[0]
                                                            for r in range(1, world)])
    assert logs.merge_parts(str(out / "log"), world) > 0
    assert len(compare_dirs(out, seq / "expected")) == 40
    assert open(name, "rb").read() == cat


@pytest.mark.timeout(600)
def test_shard_logs_merged_by_rank0(seq):
    """--shard-logs --merge-parts: rank 0 appends the parts after the last rank."""
    out = run_ranks(seq, 2, "shardmerge", ["--shard-logs", "--merge-parts"])
    assert len(compare_dirs(out, seq / "expected")) == 40


def test_rank_only_shard_logs_streams_its_part_files(seq):
    """--rank-only K --shard-logs: rank K's part files are written as its
    launches complete (no deferred rows), replace stale ones, and equal the
    default path's part files."""
    out = seq / "rankonly_parts"
    out.mkdir()
    argv = ["-f", str(SEQ["n"]), "-s", f"{SEQ['W']}x{SEQ['H']}", "-q", str(SEQ["qp"]),
            "-o", str(seq / "orig.csv"), "-r", str(seq / "recon.csv"), "-l", str(out / "log"),
            "--gpus", "2", "--rank-only", "1"]
    table = torch.load(seq / "table.pt", weights_only=True)
    names = [os.path.basename(n) for n in logs.log_names(distrun.part_prefix(str(out / "log"), 1))]
    a = distrun.parse_args(argv)
    distrun.run_rank(a, 2, 1, LookupEngine(a.W, a.H, table), torch.device("cpu"))
    placed = {n: (out / n).read_bytes() for n in names}
    for n in names:  # stale, longer than any real part
        (out / n).write_bytes(b"X" * 1_000_000)
    a = distrun.parse_args(argv + ["--shard-logs"])
    assert a.log_path == "parts"
    distrun.run_rank(a, 2, 1, LookupEngine(a.W, a.H, table), torch.device("cpu"))
    assert {n: (out / n).read_bytes() for n in names} == placed


def test_parse_args_rejects_bad_input():
    with pytest.raises(SystemExit):
        distrun.parse_args(["-f", "2", "-s", "1000x1000", "-q", "32", "-o", "a", "-r", "b"])
    with pytest.raises(SystemExit):
        distrun.parse_args(["-f", "0", "-s", "416x240", "-q", "32", "-o", "a", "-r", "b"])
    with pytest.raises(SystemExit):  # 3 pairs in 2 frames: at most 3 ranks
        distrun.parse_args(["-f", "2", "-s", "416x240", "-q", "32", "-o", "a", "-r", "b", "--gpus", "4"])
    assert distrun.parse_args(["-f", "2", "-s", "416x240", "-q", "32", "-o", "a", "-r", "b", "--gpus", "3"]).gpus == 3
    with pytest.raises(SystemExit):  # --merge-parts needs --shard-logs
        distrun.parse_args(["-f", "2", "-s", "416x240", "-q", "32", "-o", "a", "-r", "b", "--merge-parts"])
    with pytest.raises(SystemExit):
        distrun.parse_args(["-f", "2", "-s", "416x240", "-q", "32", "-o", "a", "-r", "b", "--shard-logs",
                            "--gather-records"])


def test_world_size_must_match_gpus(tmp_path):
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0",
               PYTHONPATH=os.path.join(REPO, "vvc-affine-gpu_amd"))
    r = subprocess.run([sys.executable, "-m", "vame.distrun", "-f", "2", "-s", "416x240", "-q", "32",
                        "-o", "a", "-r", "b", "--gpus", "1"], env=env, capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


# ---- MI355X: the real rank processes with the HIP engine vs the vame CLI

def run_distrun_gpu(tmp, W, H, n, qp, name, extra=(), env_extra=None):
    out = tmp / name
    out.mkdir()
    env = dict(os.environ, VAME_DIST_BACKEND="gloo", PYTHONPATH=os.path.join(REPO, "vvc-affine-gpu_amd"))
    env.update(env_extra or {})
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-m", "vame.distrun", "-f", str(n), "-s", f"{W}x{H}", "-q", str(qp),
                        "-o", str(tmp / "orig.csv"), "-r", str(tmp / "recon.csv"), "-l", str(out / "log"),
                        *extra], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return out, r.stdout


def run_cli(tmp, W, H, n, qp):
    out = tmp / "cli"
    out.mkdir()
    cli = os.path.join(REPO, "vvc-affine-gpu_amd", "bin", "vame")
    r = subprocess.run([cli, "-f", str(n), "-s", f"{W}x{H}", "-q", str(qp), "-o", str(tmp / "orig.csv"),
                        "-r", str(tmp / "recon.csv"), "-l", str(out / "log")],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:]
    return out


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("W,H,n", [(416, 240, 7), (1920, 1080, 2)])
def test_distrun_two_ranks_equals_cli(tmp_path, W, H, n):
    """`python -m vame.distrun --gpus 2` (gather and --shard-logs) writes the
    40 files of the single-process `vame` CLI byte for byte: 416x240 with 7
    POCs (POC 5 cut between the ranks), 1920x1080 with 2 POCs."""
    orig, recon = synth_sequence(W, H, n, qp=32, seed=9)
    write_csv(str(tmp_path / "orig.csv"), orig)
    write_csv(str(tmp_path / "recon.csv"), recon)
    cli = run_cli(tmp_path, W, H, n, 32)
    for name, extra in (("gather", ("--gather-records",)), ("shard", ())):
        out, stdout = run_distrun_gpu(tmp_path, W, H, n, 32, name, ("--gpus", "2", *extra))
        assert len(compare_dirs(out, cli)) == 40, name
        assert "LOG_BYTES," in stdout and '"ranks": 2' in stdout


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_distrun_forced_rccl_group_equals_cli(tmp_path):
    """`python -m vame.distrun` in a one-rank RCCL process
    group (VAME_FORCE_PG=1, backend nccl): init_process_group("nccl",
    device_id=...), the records' dist.gather into rank 0 (rank 0's own, packed
    on the GPU), all_gather_object of the timings -- and the 40 logs written
    from the gathered slab equal the single-process CLI's byte for byte
    (416x240, 7 POCs)."""
    W, H, n = 416, 240, 7
    orig, recon = synth_sequence(W, H, n, qp=32, seed=9)
    write_csv(str(tmp_path / "orig.csv"), orig)
    write_csv(str(tmp_path / "recon.csv"), recon)
    cli = run_cli(tmp_path, W, H, n, 32)
    out, stdout = run_distrun_gpu(tmp_path, W, H, n, 32, "rccl1", ("--gather-records",),
                                  {"VAME_DIST_BACKEND": "nccl", "VAME_FORCE_PG": "1"})
    assert len(compare_dirs(out, cli)) == 40
    assert '"ranks": 1' in stdout and "LOG_GATHER_TIME," in stdout


class FakeEngine:
    """Deterministic stand-in results (not the algorithm, but its record shape:
    costs below 2^31, LB = 0 for 2 CP): every record a hash of the (cur, ref,
    lambda) triple it was computed for, so a run's logs depend on
    exactly which frames each pair used -- enough to test the shard, ingest and
    log-placement plumbing at many ranks without the oracle's cost."""

    def __init__(self, W, H):
        self.n_ctus = O.lib().vame_oracle_num_ctus(W, H)

    def n_cus(self, align):
        return self.n_ctus * (284 if align else 201)

    def alloc_poc(self, nrefs, modes=3):
        return LookupEngine.alloc_poc(self, nrefs, modes)

    def affine_me_batch(self, jobs, modes, extra):
        for cur, refs, lam, out in jobs:
            for r, ref in enumerate(refs):
                h = digest(cur.numpy().view(np.uint16)) + digest(ref.numpy().view(np.uint16)) + repr(lam)
                seed = int(hashlib.sha1(h.encode()).hexdigest()[:8], 16)
                g = torch.Generator().manual_seed(seed)
                for (r2, m), (c, p) in out.items():
                    if r2 == r:
                        c.copy_(torch.randint(0, 1 << 20, c.shape, generator=g))
                        p.copy_(torch.randint(-4096, 4096, p.shape, generator=g, dtype=torch.int32))
                        p[:, 0] = 3 if m.endswith("3CP") else 2
                        if m.endswith("2CP"):  # 2-CP records carry LB = (0, 0)
                            p[:, 5:] = 0
        return [j[3] for j in jobs]


def fake_worker(rank, world, port, argv):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a = distrun.parse_args(argv)
    distrun.run_rank(a, world, rank, FakeEngine(a.W, a.H), torch.device("cpu"), dist)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(900)
def test_eight_ranks_cut_pocs_and_long_term_refs(tmp_path):
    """8 ranks over 40 frames (150 pairs): POCs 7, 16, 21, 26, 31 cut
    between ranks, long-term references of POC 8 / 16 / 24 / 32 in play, every
    rank's frames read through the shared CSV line index; both log paths equal
    a one-rank run byte for byte (the plumbing of BASELINE configs[4] at N = 8;
    stand-in results, the HIP path's parity is covered elsewhere)."""
    n = 40
    orig, recon = synth_sequence(416, 240, n, 32, seed=5)
    write_csv(str(tmp_path / "orig.csv"), orig)
    write_csv(str(tmp_path / "recon.csv"), recon)
    owners = {}
    for r in range(8):
        for p, _ in shard.pair_shard(n, 8, r):
            owners.setdefault(p, []).append(r)
    assert [p for p, o in owners.items() if len(o) > 1] == [7, 16, 21, 26, 31]

    def argv(out, *extra):
        out.mkdir()
        return ["-f", str(n), "-s", "416x240", "-q", "32", "-o", str(tmp_path / "orig.csv"),
                "-r", str(tmp_path / "recon.csv"), "-l", str(out / "log"), "--modes", "2cp", *extra]
    one = tmp_path / "one"
    a = distrun.parse_args(argv(one))
    distrun.run_rank(a, 1, 0, FakeEngine(416, 240), torch.device("cpu"))
    from vame.launch import free_port
    for name, extra in (("gather8", ("--gather-records",)), ("shard8", ())):
        mp.spawn(fake_worker, args=(8, free_port(), argv(tmp_path / name, *extra)), nprocs=8, join=True)
        assert len(compare_dirs(tmp_path / name, one)) == 20, name
