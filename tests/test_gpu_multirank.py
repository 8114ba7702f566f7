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
    # slabs of one or two planes (400 / 800 nodes): a slab's ids span one or two 1024-id list
    # tiles, so an exchange region may hold no tile at all
    (8000, "Imp3D", "push-sum", 4, 300, 100, 16),
    (8000, "Imp3D", "gossip", 5, 600, 200, 16),
    (27000, "Imp3D", "push-sum", 12, 300, 100, 5),
    (216000, "3D", "push-sum", 9, 200, 75, 2),
    (27000, "3D", "gossip", 4, 2000, 500, 3),
    (5000, "line", "gossip", 6, 8000, 2000, 2),
    (777, "line", "push-sum", 2, 1500, 500, 4),
    (30000, "full", "push-sum", 8, 300, 50, 2),
    (20000, "full", "push-sum", 5, 120, 40, 3),
    (50000, "full", "gossip", 3, 400, 100, 3),
    (3000, "full", "gossip", 9, 2000, 400, 2),
]


@pytest.mark.parametrize("kernel", ["default", "tile", "col", "regions"])
@pytest.mark.parametrize("n,topo,alg,seed,rounds,chk,ranks", CASES, ids=lambda v: str(v))
def test_virtual_ranks_parity(kernel, n, topo, alg, seed, rounds, chk, ranks, monkeypatch):
    """default: the product library's own kernel choice; the others force a
    variant through the experiments build (GP_KERNEL).  regions: Imp3D push-sum
    with the round kernel run region by region (GP_RREGIONS=1; the product does
    so for slabs of >= 2^24 nodes, gp_api.hip round_regions) -- four launches per
    round, the lists of each region sent behind the next, the receive buffer by
    round parity, regions holding no plane at 8 000 nodes / 16 ranks."""
    if kernel == "col" and (topo == "line" or alg == "push-sum"):
        pytest.skip("the column march runs lattice gossip only")
    if topo == "full" and kernel not in ("default", "tile"):
        pytest.skip("the full topology has one kernel set")
    if kernel == "regions" and (topo, alg) != ("Imp3D", "push-sum"):
        pytest.skip("region rounds: Imp3D push-sum across ranks")
    exp = kernel != "default"
    if kernel == "regions":
        monkeypatch.setenv("GP_RREGIONS", "1")
        monkeypatch.setenv("GP_WALK", "3")  # (the product walks the per-XCD queues from g / W >= 64)
        monkeypatch.setenv("GP_CHECK_CLOSE", "1")
    elif exp:
        monkeypatch.setenv("GP_KERNEL", kernel)
        monkeypatch.setenv("GP_CHECK_CLOSE", "1")  # alerts recounted from the state after every batch
    sim = Sim(n, topo, alg, seed=seed, virtual_ranks=ranks, experimental=exp)
    orc = Oracle(n, topo, alg, seed)
    assert sim.info().num_gpus == ranks
    if kernel == "regions":
        assert sim._L.gp_debug_round_regions(sim._h) > 1
    elif topo == "Imp3D" and alg == "push-sum":
        assert (sim._L.gp_debug_round_regions(sim._h) if exp else 1) == 1  # small slabs: one launch
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


def test_region_rounds_kernel_timing(monkeypatch):
    """Kernel timing with the round kernel run region by region: one entry per round, the sum
    of its region launches (events around each launch; the packs between them excluded)."""
    monkeypatch.setenv("GP_RREGIONS", "1")
    monkeypatch.setenv("GP_WALK", "3")
    sim = Sim(64000, "Imp3D", "push-sum", seed=5, virtual_ranks=2, experimental=True, kernel_timing=True)
    assert sim._L.gp_debug_round_regions(sim._h) > 1
    sim.step(20)
    sim.kernel_stats(reset=True)
    assert len(sim.step(30)) == 30
    ms, n, name = sim.kernel_stats()
    assert n == 30 and ms > 0 and "tile" in name
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


@pytest.mark.parametrize("topo,alg", [("Imp3D", "push-sum"), ("Imp3D", "gossip"), ("full", "push-sum"),
                                      ("full", "gossip")])
def test_exchange_overflow_fails_every_rank(topo, alg, monkeypatch):
    """An exchange buffer that overflows invalidates the round on every rank: the
    flag is summed over ranks with the round's bookkeeping, so gp_step fails with
    GP_ESTATE (never silently truncated messages).  GP_XCAP (experiments build)
    caps every per-pair buffer at a few entries to force it."""
    from gossipprotocol_amd._lib import GossipError
    monkeypatch.setenv("GP_XCAP", "2")
    sim = Sim(64000, topo, alg, seed=5, virtual_ranks=3, experimental=True)
    with pytest.raises(GossipError) as e:
        sim.step(200)
    assert e.value.code == -5 and "overflow" in str(e.value)
    sim.close()


@pytest.mark.parametrize("topo,alg", [("Imp3D", "push-sum"), ("Imp3D", "gossip"), ("full", "push-sum")])
def test_virtual_ranks_max_world(topo, alg):
    """The largest world the exchange supports (XMAXW = 16, gp_xchg.hpp): every rank,
    rank 15 included, receives its random-edge / full messages (k_pack keeps a
    destination rank in 4 bits; the "no message" value is the sender's own rank)."""
    n, seed, rounds = 32768, 11, 400
    sim = Sim(n, topo, alg, seed=seed, virtual_ranks=16)
    orc = Oracle(n, topo, alg, seed)
    assert sim.info().num_gpus == 16
    done = 0
    while done < rounds:
        ga, oa = sim.step(100), orc.step(100)
        assert ga == oa, f"alerts differ in rounds {done}..{done + 100}"
        same_state(alg, sim.state(), orc.state())
        done += 100
        if len(ga) < 100:
            break
    sim.close()
    orc.close()


@pytest.mark.parametrize("ranks", [1, 3])
def test_col_gossip_byte_counters(ranks, monkeypatch):
    """Imp3D gossip on the column kernel with the random-edge delivery counts held
    as bytes, four per word (GP_RQ8=1, experiments build): local senders' atomics,
    the exchange's counts and the seed's round-0 send all add into byte lanes --
    bit-exact vs the oracle on one and on three ranks."""
    monkeypatch.setenv("GP_KERNEL", "col")
    monkeypatch.setenv("GP_RQ8", "1")
    n, seed = 125000, 12
    sim = Sim(n, "Imp3D", "gossip", seed=seed, virtual_ranks=ranks, experimental=True)
    orc = Oracle(n, "Imp3D", "gossip", seed)
    for _ in range(3):
        ga, oa = sim.step(100), orc.step(100)
        assert ga == oa
        same_state("gossip", sim.state(), orc.state())
    sim.close()
    orc.close()
