"""bench.py's multi-rank contract: `--gpus N` without a
launcher starts N ranks itself; under a launcher, WORLD_SIZE must equal --gpus.
The argument checks run before anything touches a GPU (CPU tests); the 2-rank
run itself needs the MI355X (gloo: both ranks share the test box's one GPU)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(args, env=None, timeout=60):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=e,
                          capture_output=True, text=True, timeout=timeout)


def test_world_size_must_match_gpus():
    r = run_bench(["--gpus", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr and "--gpus 1" in r.stderr
    assert r.stdout == ""


def test_gpus_must_be_positive():
    r = run_bench(["--gpus", "0"])
    assert r.returncode != 0 and "--gpus" in r.stderr


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("weak", ["streams", "sequence"])
def test_bench_gpus2_launches_two_ranks(weak):
    """`python bench.py --gpus 2 --config c2 --steps 3` with no launcher: two
    ranks (gloo, one GPU), one JSON line from rank 0 with n_gpus 2, the world
    it ran in, and the gathered records byte-identical to rank 0's recompute
    (both weak-scaling forms: a sequence per rank, pair blocks of one)."""
    r = run_bench(["--gpus", "2", "--config", "c2", "--steps", "3", "--warmup", "1",
                   "--no-cpu-baseline", "--weak", weak], {"VAME_DIST_BACKEND": "gloo"}, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["world"] == {"size": 2, "backend": "gloo", "launcher": "bench.py"}
    assert d["config"]["rows_per_step_all"] == 2 * d["config"]["rows_per_step_rank0"]
    assert d["gather"]["check"]["byte_identical"] is True
    assert d["step_ms"]["min"] <= d["step_ms"]["median"] <= d["step_ms"]["max"]
    assert d["config"]["pairs_per_step_rank0"] == 3
    assert d["gather"]["check"]["cut_pocs"] == []  # sequence: POC 1-2 | POC 3, no cut
    assert d["config"]["parallelism"].endswith("(a sequence of its own per rank)" if weak == "streams"
                                               else "(pair_shard of one sequence)")


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_bench_under_torchrun():
    """The driver's multi-GPU command form: `python -m torch.distributed.run
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P
    bench.py --gpus 2 ...` (gloo here: both ranks share the test box's GPU).
    The launcher set WORLD_SIZE, so bench.py starts no ranks of its own."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    e = dict(os.environ, VAME_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "VAME_LAUNCHER"):
        e.pop(k, None)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port),
                        os.path.join(REPO, "bench.py"), "--gpus", "2", "--config", "c2", "--steps", "3",
                        "--warmup", "1", "--no-cpu-baseline"], env=e, capture_output=True, text=True,
                       timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["world"] == {"size": 2, "backend": "gloo", "launcher": "external"}
    assert d["gather"]["check"]["byte_identical"] is True
    assert d["native"]["lib"].endswith("libvame.so")
