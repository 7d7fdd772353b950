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


POISON = """
import sys, torch
def boom(*a, **k):
    raise RuntimeError("torch.cuda touched in the launcher parent")
for name in ("device_count", "is_available", "init", "set_device", "current_device", "_lazy_init",
             "synchronize", "get_device_properties"):
    setattr(torch.cuda, name, boom)
sys.path.insert(0, {pkg!r})
from vame.launch import launch_ranks
rc = launch_ranks(2, ["-c", "import os, sys; sys.exit(0 if os.environ['WORLD_SIZE'] == '2' and "
                            "os.environ['LOCAL_RANK'] in ('0', '1') else 3)"], "nccl", "poison-test")
sys.exit(rc)
"""


def fake_topology(root, gpus, cpus=1):
    """A KFD topology tree: CPU nodes (gpu_id 0) then GPU nodes."""
    for k in range(cpus + gpus):
        d = root / str(k)
        d.mkdir()
        (d / "gpu_id").write_text("0\n" if k < cpus else f"{1000 + k}\n")
    return str(root)


def test_launcher_never_touches_torch_cuda(tmp_path):
    """the nccl branch of launch_ranks must not initialise
    the GPU runtime in the parent that spawns the ranks.  Every torch.cuda
    entry point raises in this parent; the 2 ranks start and exit 0 (with a
    fake 2-GPU topology, and with none at all)."""
    pkg = os.path.join(REPO, "vvc-affine-gpu_amd")
    code = POISON.format(pkg=pkg)
    for env in ({"VAME_KFD_TOPOLOGY": fake_topology(tmp_path, 2)},
                {"VAME_KFD_TOPOLOGY": str(tmp_path / "absent")}):
        r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **env),
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        assert "touched" not in r.stderr


def test_launcher_refuses_more_ranks_than_gpus(tmp_path):
    pkg = os.path.join(REPO, "vvc-affine-gpu_amd")
    code = POISON.format(pkg=pkg)
    r = subprocess.run([sys.executable, "-c", code],
                       env=dict(os.environ, VAME_KFD_TOPOLOGY=fake_topology(tmp_path, 1)),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "2 ranks but 1 GPUs visible" in r.stderr


def test_visible_gpu_count(tmp_path, monkeypatch):
    from vame.launch import visible_gpu_count
    topo = fake_topology(tmp_path, 8, cpus=2)
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    assert visible_gpu_count(topo) == 8
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "3,5")
    assert visible_gpu_count(topo) == 2
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "1")
    assert visible_gpu_count(topo) == 1
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES")
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")  # empty: no restriction
    assert visible_gpu_count(topo) == 8
    assert visible_gpu_count(str(tmp_path / "none")) is None


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_bench_forced_rccl_group():
    """the RCCL branch on one MI355X.  VAME_FORCE_PG=1 forms
    a real one-rank nccl process group, so init_process_group("nccl",
    device_id=...), the device-tensor all_reduce of the timing and the
    dist.gather of the decision records into rank 0 all run through RCCL;
    rank 0 then recomputes its block and checks the gathered records."""
    r = run_bench(["--config", "c2", "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--fs-frames", "4"],
                  {"VAME_FORCE_PG": "1"}, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["world"]["backend"] == "nccl" and d["world"]["forced_pg"] is True and d["world"]["size"] == 1
    assert d["gather"]["backend"] == "nccl"
    assert d["gather"]["check"]["byte_identical"] is True and len(d["gather"]["check"]["pocs"]) >= 1
    assert d["n_gpus"] == 1 and d["scaling_form"] == "streams"
    check_frame_shard(d, 1, "nccl")


def check_frame_shard(d, world, backend):
    """The `frame_shard` record: one 2160p sequence cut into
    pair blocks over the ranks, the gather into rank 0 inside the timed span,
    rank 0's recompute check byte-identical."""
    fs = d["frame_shard"]
    assert fs["backend"] == backend and fs["check"]["byte_identical"] is True
    assert fs["pairs"] == sum(min(4, p) for p in range(1, fs["frames"] + 1))
    assert fs["ms"] >= fs["kernel_ms"]["max"] >= fs["kernel_ms"]["min"] > 0
    assert fs["rows"] == fs["pairs"] * 494700 and fs["rows_per_s"] > 0
    assert fs["exchange_ms"] >= 0 and fs["gather_ms_max"] >= 0
    # every rank's slab is padded to the largest block's words: compact records
    # of 20 (2-CP) + 28 (3-CP) bytes per candidate CU (247,350 per CP mode at
    # 2160p), from every rank but rank 0
    per_pair = 247350 * (20 + 28)
    if world == 1:
        assert fs["bytes_into_rank0"] == 0
    else:
        assert fs["bytes_into_rank0"] == (world - 1) * -(-fs["pairs"] // world) * per_pair


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("weak", ["streams", "sequence"])
def test_bench_gpus2_launches_two_ranks(weak):
    """`python bench.py --gpus 2 --config c2 --steps 3` with no launcher: two
    ranks (gloo, one GPU), one JSON line from rank 0 with n_gpus 2, the world
    it ran in, and the gathered records byte-identical to rank 0's recompute
    (both weak-scaling forms: a sequence per rank, pair blocks of one)."""
    r = run_bench(["--gpus", "2", "--config", "c2", "--steps", "3", "--warmup", "1",
                   "--no-cpu-baseline", "--weak", weak, "--fs-frames", "6" if weak == "streams" else "0"],
                  {"VAME_DIST_BACKEND": "gloo"}, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["world"] == {"size": 2, "backend": "gloo", "launcher": "bench.py",
                                               "forced_pg": False}
    assert d["config"]["rows_per_step_all"] == 2 * d["config"]["rows_per_step_rank0"]
    assert d["gather"]["check"]["byte_identical"] is True
    assert d["step_ms"]["min"] <= d["step_ms"]["median"] <= d["step_ms"]["max"]
    assert d["config"]["pairs_per_step_rank0"] == 3
    assert d["gather"]["check"]["cut_pocs"] == []  # sequence: POC 1-2 | POC 3, no cut
    assert d["config"]["parallelism"].endswith("(a sequence of its own per rank)" if weak == "streams"
                                               else "(pair_shard of one sequence)")
    if weak == "streams":  # POC 1-6 = 18 pairs, 9 per rank: POC 4 cut between the ranks
        check_frame_shard(d, 2, "gloo")
        assert d["frame_shard"]["check"]["cut_pocs"] == [4]
    else:
        assert "frame_shard" not in d
    g = d["gather"]  # pack and exchange timed apart
    assert g["pack_ms"] >= 0 and g["exchange_ms"] >= 0 and g["bytes_into_rank0"] > 0


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
                        "--warmup", "1", "--no-cpu-baseline", "--fs-frames", "0"], env=e, capture_output=True, text=True,
                       timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["world"] == {"size": 2, "backend": "gloo", "launcher": "external",
                                               "forced_pg": False}
    assert d["gather"]["check"]["byte_identical"] is True
    assert d["native"]["lib"].endswith("libvame.so")
