"""One process per GPU: start the ranks of a frame-sharded run
without an external launcher, and join the process group inside a rank.

`launch_ranks` re-runs the calling script as N child processes with RANK /
LOCAL_RANK / WORLD_SIZE / MASTER_* set (rendezvous on 127.0.0.1).  It must run
before anything in the parent touches the GPU (counting devices does not).
`init_rank` joins: backend nccl (RCCL over xGMI, rank r on GPU r) or, with
VAME_DIST_BACKEND=gloo, the CPU rehearsal of several ranks sharing the GPUs.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv: list[str], backend: str, tag: str) -> int:
    """Run `python argv...` as ranks 0..n-1 and wait.  If a rank fails, the
    others are stopped (they would wait in a collective forever).  Returns
    the exit code (0 when every rank succeeded)."""
    import torch
    if backend == "nccl" and torch.cuda.device_count() < n:
        print(f"{tag}: {n} ranks but {torch.cuda.device_count()} GPUs visible", file=sys.stderr)
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


def init_rank(world: int, backend: str):
    """Join the process group of a `world`-rank run; returns (dist module or
    None, rank, torch device).  gloo ranks share the visible GPUs round-robin."""
    import torch
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1:
        torch.cuda.set_device(0)
        return None, 0, torch.device("cuda", 0)
    import torch.distributed as dist
    local = local % torch.cuda.device_count() if backend != "nccl" else local
    torch.cuda.set_device(local)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    if dist.get_world_size() != world:
        raise SystemExit(f"world size {dist.get_world_size()} != {world}")
    return dist, rank, torch.device("cuda", local)
