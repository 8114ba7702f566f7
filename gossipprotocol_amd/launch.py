"""Rank-process launcher for one-process-per-GPU runs.

The reference is one process (`dotnet run`, Program.fs:31-34); the multi-GPU
path is one process per GPU with RCCL between them.  `run_ranks` starts the N
rank processes of a command *before anything touches a GPU* (this module never
loads libgossip_hip or torch: a process that has initialised the GPU must not
spawn GPU work by exec), waits for all of them, and turns the first failure into
the launcher's exit status after stopping the other ranks -- a request for N GPUs
never silently runs on fewer.  Used by bench.py and `python -m gossipprotocol_amd
--gpus N`; the C++ CLI (`gossip --gpus N`, csrc/gossip_cli.cpp) does the same
with fork.

Every rank gets RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT (for a
torch.distributed group, as torch.distributed.run would set) and GOSSIP_RDV, a
fresh file path for gp_rendezvous_id (rank 0's RCCL id).
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import shutil
import signal
import socket
import subprocess
import sys
import tempfile
import time


@contextlib.contextmanager
def stdout_to_stderr():
    """Route file descriptor 1 to stderr for the duration (RCCL prints its version
    line on stdout when a communicator starts; stdout is the reference's contract
    / bench.py's one JSON line).  C stdio is flushed on both edges."""
    libc = ctypes.CDLL(None)
    sys.stdout.flush()
    libc.fflush(None)
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        sys.stdout.flush()
        libc.fflush(None)
        os.dup2(saved, 1)
        os.close(saved)


def free_port() -> int:
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def rehearsal_env(rank: int, tag: str = "gp-rehearsal") -> dict:
    """All ranks on one GPU (a one-GPU box): RCCL refuses two ranks of one
    communicator on one device of one host, so each rank claims a host id of its
    own and the ranks talk over RCCL's socket transport on loopback."""
    return {"NCCL_HOSTID": f"{tag}-{os.getpid()}-{rank}", "NCCL_SOCKET_IFNAME": os.environ.get("NCCL_SOCKET_IFNAME", "lo"),
            "NCCL_IB_DISABLE": os.environ.get("NCCL_IB_DISABLE", "1")}


def run_ranks(cmd, world: int, env_for_rank=None, log=None, poll_s: float = 0.2, ok_codes=(0,)) -> int:
    """Run `cmd` (argv list) as `world` rank processes; return the first failing
    exit code (>= 1) or rank 0's.  env_for_rank(r) -> extra environment of rank r.
    ok_codes: exit codes that are results, not failures (the CLI's 3 = not converged)."""
    log = log or (lambda *a: print(*a, file=sys.stderr, flush=True))
    rdv_dir = tempfile.mkdtemp(prefix="gossip_rdv_", dir=os.environ.get("TMPDIR", "/tmp"))
    port = free_port()
    nonce = os.urandom(8).hex()  # this launch's rendezvous nonce (gp_rendezvous_id)
    procs = []
    failed = None
    try:
        for r in range(world):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GOSSIP_RDV=os.path.join(rdv_dir, "rccl_id"),
                       GOSSIP_RDV_NONCE=nonce, GOSSIP_LAUNCHED="1")
            if env_for_rank is not None:
                env.update(env_for_rank(r))
            procs.append(subprocess.Popen(cmd, env=env, start_new_session=True))
        while True:
            for r, p in enumerate(procs):
                rc = p.poll()
                if rc is not None and rc not in ok_codes and failed is None:
                    failed = (r, rc)
            if failed is not None or all(p.poll() is not None for p in procs):
                break
            time.sleep(poll_s)
    finally:
        if failed is not None:
            log(f"[launch] rank {failed[0]} of {world} failed (exit {failed[1]}); stopping the other ranks")
        for sig, wait in ((signal.SIGTERM, 10.0), (signal.SIGKILL, 30.0)):
            live = [p for p in procs if p.poll() is None]
            if not live:
                break
            for p in live:
                try:
                    os.killpg(p.pid, sig)  # the rank's own process group (start_new_session)
                except ProcessLookupError:
                    pass
            t0 = time.perf_counter()
            while any(p.poll() is None for p in live) and time.perf_counter() - t0 < wait:
                time.sleep(0.1)
        shutil.rmtree(rdv_dir, ignore_errors=True)
    if failed is not None:
        return failed[1] if failed[1] > 0 else 1
    return procs[0].returncode
