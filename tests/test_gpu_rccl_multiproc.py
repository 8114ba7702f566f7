"""GPU: the one-process-per-GPU RCCL path with world > 1, as separate processes.

The test box has one GPU, and RCCL refuses two ranks of one communicator on one
device of one host ("Duplicate GPU detected").  Giving every rank
its own NCCL_HOSTID makes RCCL treat the processes as different hosts, so the
ranks share the one MI355X and talk over RCCL's socket transport on loopback.
Everything above the transport is the multi-GPU product path: gp_create_rank ->
ncclCommInitRank, the slab plan, the grouped ncclSend/ncclRecv halo and random-
edge exchange (full push-sum: two halves on the exchange stream), and the
ncclAllReduce of the round bookkeeping -- only xGMI P2P is replaced by sockets.

Each case runs W worker processes (tests/helpers/rccl_worker.py) and requires
the per-round alert counts and every rank's slab state (c, s, w, flags) to equal
a single-process run bit for bit (single-process runs are oracle-checked in
test_gpu_parity.py).  Reference semantics: Program.fs:51-56 (alert count),
101-131 / 209-216 (deliveries) via SRS v1.
"""
import os
import socket
import subprocess
import sys
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "helpers", "rccl_worker.py")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_ranks(world, n, topo, alg, seed, rounds, timeout=150):
    """Start `world` rank processes on device 0, wait for all, return their npz records."""
    out = tempfile.mkdtemp(prefix="gp_rccl_mp_")
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GP_BENCH_DEVICE="0",
                   NCCL_HOSTID=f"gp-rehearsal-{r}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1",
                   HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, "-u", WORKER, out, str(n), topo, alg, str(seed), str(rounds)],
                                      env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      start_new_session=True))
    logs, codes = [], []
    try:
        for p in procs:
            o, _ = p.communicate(timeout=timeout)
            logs.append(o.decode(errors="replace")[-3000:])
            codes.append(p.returncode)
    finally:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, 9)
                p.wait()
    assert codes == [0] * world, "rank processes failed:\n" + "\n----\n".join(logs)
    return [dict(np.load(os.path.join(out, f"rank{r}.npz"))) for r in range(world)]


CASES = [
    (2, 27000, "Imp3D", "push-sum", 3, 160),
    (3, 27000, "Imp3D", "push-sum", 5, 120),
    (2, 20000, "full", "push-sum", 2, 40),
    (2, 27000, "Imp3D", "gossip", 4, 300),
    (2, 27000, "3D", "push-sum", 6, 200),
    (2, 2000, "line", "gossip", 7, 300),
    (4, 64000, "Imp3D", "push-sum", 8, 120),
    (4, 40000, "full", "push-sum", 9, 30),
    (2, 200**3, "Imp3D", "gossip", 4, 150),  # g = 200: the column kernel, random-edge counts through the exchange
    (3, 200**3, "Imp3D", "gossip", 6, 120),
]


@pytest.mark.parametrize("world,n,topo,alg,seed,rounds", CASES)
def test_rccl_processes_match_single(world, n, topo, alg, seed, rounds):
    from gossipprotocol_amd import Simulation
    recs = run_ranks(world, n, topo, alg, seed, rounds)
    with Simulation(n, topo, alg, seed=seed) as ref:
        want = ref.step(rounds)
        info = ref.info()
        full = ref.state()
    for r, rec in enumerate(recs):
        assert list(rec["alerts"]) == want, f"rank {r}: per-round alert counts differ"
        assert int(rec["rounds"]) == info.rounds
        assert int(rec["alerts_total"]) == info.alerts_total
        lo = int(rec["first"])
        cnt = len(rec["c"])
        for k in ("c", "s", "w", "flags"):
            np.testing.assert_array_equal(rec[k], full[k][lo:lo + cnt], err_msg=f"rank {r} slab [{lo}, +{cnt}) {k}")
    # the slabs tile the id range
    firsts = sorted((int(rec["first"]), len(rec["c"])) for rec in recs)
    assert firsts[0][0] == 0 and sum(c for _, c in firsts) == info.population
    assert all(a + c == b for (a, c), (b, _) in zip(firsts, firsts[1:]))


@pytest.mark.parametrize("world,n,topo,alg,rounds", [
    # the BASELINE configurations that shard, each as two rank processes at its full size, in the
    # default -m gpu suite (~70 s together), so the driver's own run sees them bit-exact
    (2, 10**9, "Imp3D", "push-sum", 140),   # C5, the headline: past activation into steady state
    (2, 10**8, "full", "push-sum", 60),     # C4: the two-half exchange
    (2, 10**8, "Imp3D", "gossip", 100),     # C3: counts as bitmaps + halo planes
])
def test_rccl_processes_baseline_size(world, n, topo, alg, rounds):
    """BASELINE configurations as rank processes: per-round alerts and an xxh3-128 digest of every
    rank's slab equal the single-process run's."""
    sys.path.insert(0, os.path.join(ROOT, "tests", "helpers"))
    from rccl_worker import slab_digest
    from gossipprotocol_amd import Simulation
    recs = run_ranks(world, n, topo, alg, 1, rounds, timeout=900)
    with Simulation(n, topo, alg, seed=1) as ref:
        want = ref.step(rounds)
        info = ref.info()
        if alg == "push-sum" and topo == "Imp3D":
            assert info.active == info.population, "steady state not reached inside the window"
        for r, rec in enumerate(recs):
            assert list(rec["alerts"]) == want
            lo, cnt = int(rec["first"]), int(rec["count"])
            assert str(rec["digest"]) == slab_digest(ref, lo, cnt), f"rank {r} slab [{lo}, +{cnt}) differs"
