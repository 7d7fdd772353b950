"""One process per GPU: start the ranks of a frame-sharded run
without an external launcher, and join the process group inside a rank.

`launch_ranks` re-runs the calling script as N child processes with RANK /
LOCAL_RANK / WORLD_SIZE / MASTER_* set (rendezvous on 127.0.0.1).  It must run
before anything in the parent touches the GPU, and it never calls torch.cuda
or HIP itself: the GPUs are counted from the KFD topology in sysfs
(`visible_gpu_count`), and when that count is unknown each rank checks its own
LOCAL_RANK against the GPUs it sees (`init_rank`).
`init_rank` joins: backend nccl (RCCL over xGMI, rank r on GPU r) or, with
VAME_DIST_BACKEND=gloo, the CPU rehearsal of several ranks sharing the GPUs.
VAME_FORCE_PG=1 makes a one-rank run form a real one-rank process group too,
so the collective code of an N-GPU run (init_process_group("nccl",
device_id=...), device all_reduce, the gather into rank 0) executes on a
single GPU.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time

KFD_TOPOLOGY = "/sys/class/kfd/kfd/topology/nodes"


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def visible_gpu_count(topology: str | None = None) -> int | None:
    """GPUs this process could use, counted without touching the GPU runtime:
    KFD topology nodes with a non-zero gpu_id (CPU nodes have gpu_id 0),
    narrowed by ROCR_VISIBLE_DEVICES, then HIP_VISIBLE_DEVICES /
    CUDA_VISIBLE_DEVICES (comma-separated lists).  None when the topology is
    not readable (no KFD here): the ranks then check for themselves."""
    topology = topology or os.environ.get("VAME_KFD_TOPOLOGY", KFD_TOPOLOGY)
    try:
        nodes = os.listdir(topology)
    except OSError:
        return None
    n = 0
    for node in nodes:
        try:
            with open(os.path.join(topology, node, "gpu_id")) as f:
                n += int(f.read().strip() or "0") != 0
        except (OSError, ValueError):
            continue
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v:  # unset or empty: no restriction
            n = min(n, len([t for t in v.split(",") if t.strip()]))
    return n


def launch_ranks(n: int, argv: list[str], backend: str, tag: str) -> int:
    """Run `python argv...` as ranks 0..n-1 and wait.  If a rank fails, the
    others are stopped (they would wait in a collective forever).  Returns
    the exit code (0 when every rank succeeded).  Touches no GPU API."""
    if backend == "nccl":
        vis = visible_gpu_count()
        if vis is not None and vis < n:
            print(f"{tag}: {n} ranks but {vis} GPUs visible", file=sys.stderr)
            return 2
    port = free_port()
    pkg = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # `import vame` in the ranks
    path = os.pathsep.join([pkg] + [p for p in [os.environ.get("PYTHONPATH")] if p])
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   VAME_LAUNCHER=tag, PYTHONPATH=path)
        procs.append(subprocess.Popen([sys.executable] + argv, env=env))
    rc = 0
    while procs:
        for p in list(procs):
            c = p.poll()
            if c is None:
                continue
            procs.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 1
                for q in procs:  # the exact children started above
                    q.terminate()
        time.sleep(0.05)
    return rc


def forced_pg() -> bool:
    """VAME_FORCE_PG=1: a one-rank run joins a one-rank process group."""
    return os.environ.get("VAME_FORCE_PG", "") == "1"


def init_rank(world: int, backend: str):
    """Join the process group of a `world`-rank run; returns (dist module or
    None, rank, torch device).  gloo ranks share the visible GPUs round-robin;
    an nccl rank whose LOCAL_RANK has no GPU exits non-zero (launch_ranks then
    stops the others).  A one-rank run has no process group unless
    VAME_FORCE_PG=1, which forms a real one of size 1 (env:// rendezvous on
    127.0.0.1, as the launcher's ranks do)."""
    import torch
    if world == 1 and not forced_pg():
        torch.cuda.set_device(0)
        return None, 0, torch.device("cuda", 0)
    if world == 1:
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("LOCAL_RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(free_port()))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch.distributed as dist
    ndev = torch.cuda.device_count()
    if backend == "nccl":
        if local >= ndev:
            raise SystemExit(f"rank {rank}: LOCAL_RANK {local} but {ndev} GPUs visible")
    else:
        local = local % ndev
    torch.cuda.set_device(local)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    if dist.get_world_size() != world:
        raise SystemExit(f"world size {dist.get_world_size()} != {world}")
    return dist, rank, torch.device("cuda", local)
