"""GPU: the multi-GPU path (slabs, halo planes, random-edge exchange, rank-sum
bookkeeping) run as in-process virtual ranks on one MI355X, bit-exact against
the single-rank CPU oracle.  The RCCL transport moves the same buffers between
processes; its launch path is covered by tests/test_multirank_gloo.py (plan)
and the driver's multi-GPU bench."""
import numpy as np
import pytest

from tests.oracle_ctypes import Oracle

pytestmark = pytest.mark.gpu


def Sim(*a, **k):
    from gossipprotocol_amd import Simulation
    return Simulation(*a, **k)


def same_state(alg, gs, os_):
    if alg == "gossip":
        np.testing.assert_array_equal(gs["c"], os_["c"])
    else:
        np.testing.assert_array_equal(gs["s"], os_["s"])
        np.testing.assert_array_equal(gs["w"], os_["w"])
    np.testing.assert_array_equal(gs["flags"], os_["flags"])


CASES = [  # (num_nodes, topology, algorithm, seed, rounds, checkpoint, ranks)
    (64000, "Imp3D", "push-sum", 5, 300, 97, 2),
    (64000, "Imp3D", "push-sum", 6, 200, 50, 3),
    (125000, "Imp3D", "gossip", 7, 300, 101, 4),
    (27000, "Imp3D", "gossip", 3, 2000, 400, 2),
    (216000, "3D", "push-sum", 9, 200, 75, 2),
    (27000, "3D", "gossip", 4, 2000, 500, 3),
    (5000, "line", "gossip", 6, 8000, 2000, 2),
    (777, "line", "push-sum", 2, 1500, 500, 4),
    (30000, "full", "push-sum", 8, 300, 50, 2),
    (20000, "full", "push-sum", 5, 120, 40, 3),
    (50000, "full", "gossip", 3, 400, 100, 3),
    (3000, "full", "gossip", 9, 2000, 400, 2),
]


@pytest.mark.parametrize("kernel", ["tile", "tile2", "xtile", "wave", "col"])
@pytest.mark.parametrize("n,topo,alg,seed,rounds,chk,ranks", CASES, ids=lambda v: str(v))
def test_virtual_ranks_parity(kernel, n, topo, alg, seed, rounds, chk, ranks, monkeypatch):
    if kernel in ("col", "xtile") and topo == "line":
        pytest.skip("lattice kernel")
    if topo == "full" and kernel != "tile":
        pytest.skip("the full topology has one kernel set")
    monkeypatch.setenv("GP_KERNEL", kernel)
    sim, orc = Sim(n, topo, alg, seed=seed, virtual_ranks=ranks), Oracle(n, topo, alg, seed)
    assert sim.info().num_gpus == ranks
    done = 0
    while done < rounds:
        k = min(chk, rounds - done)
        ga, oa = sim.step(k), orc.step(k)
        assert ga == oa, f"alerts differ in rounds {done}..{done + k}"
        same_state(alg, sim.state(), orc.state())
        done += k
        if len(ga) < k:
            break
    assert sim.rounds == orc.rounds and sim.alerts_total == orc.alerts_total
    sim.close()


@pytest.mark.parametrize("topo", ["Imp3D", "full"])
def test_virtual_ranks_converge_like_single(topo):
    """Whole runs to convergence: same round count and alert sequence for 1, 2, 4, 8 ranks."""
    ref = None
    for ranks in (1, 2, 4, 8):
        sim = Sim(8000, topo, "push-sum", seed=3, virtual_ranks=ranks)
        alerts = sim.step(100000)
        st = sim.state()
        key = (sim.rounds, tuple(alerts), st["s"].tobytes(), st["w"].tobytes())
        if ref is None:
            ref = key
        assert key == ref, f"{ranks} ranks differ from 1 rank"
        sim.close()
