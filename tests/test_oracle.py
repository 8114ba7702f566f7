"""CPU tests: the oracles against known answers, each other and the golden fixtures.

Pins: Philox4x32-10 Random123 KATs; neighbour orders from
a literal transliteration of Program.fs:180-261 (oracle/srs_py.py); the C
oracle against the independent Python restatement; both against the committed
golden fixtures.  Reference-output parity is "parity unpinned" (no runnable
reference, no reference fixtures).
"""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import srs_py
from tests.oracle_ctypes import Oracle, lib, philox

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "srs_v1_golden.json")

KATS = [  # Random123 published Philox4x32-10 vectors
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,want", KATS)
def test_philox_kat(ctr, key, want):
    assert philox(ctr, key) == want
    assert srs_py.philox4x32_10(ctr, key) == want


def test_uniform_c_vs_python():
    rng = np.random.default_rng(7)
    for _ in range(2000):
        seed = int(rng.integers(0, 2**63))
        stream = int(rng.integers(0, 5))
        node = int(rng.integers(0, 2**32))
        rnd = int(rng.integers(0, 2**32))
        m = int(rng.integers(0, 2**32))
        assert lib().or_uniform(seed, stream, node, rnd, m) == srs_py.uniform(seed, stream, node, rnd, m)
    assert srs_py.uniform(1, 0, 5, 0, 0) == 0  # U(0) = 0 (Random().Next(0, 0) returns 0)


def test_icbrt_exact():
    for g in list(range(0, 3000)) + [465, 1000, 1625]:
        n = g ** 3
        assert lib().or_icbrt_ceil(n) == g == srs_py.icbrt_ceil(n)
        if g > 1:
            assert lib().or_icbrt_ceil(n - 1) == g
            assert lib().or_icbrt_ceil(n + 1) == g + 1
    # the libm trap of Program.fs:239 (Q3): cbrt(27.0) is not exactly 3 on glibc
    assert srs_py.icbrt_ceil(27) == 3


@pytest.mark.parametrize("n,topo,P,T,g", [
    (1000, "line", 1001, 1000, 0), (10**6, "3D", 10**6, 10**6, 100),
    (10**8, "Imp3D", 100544625, 100544625, 465), (10**8, "full", 100000001, 10**8, 0),
    (10**9, "Imp3D", 10**9, 10**9, 1000), (9000, "3D", 9261, 9261, 21),
])
def test_resolve_configs(n, topo, P, T, g):
    assert srs_py.resolve(n, topo) == (P, T, g)


@pytest.mark.parametrize("n,topo", [(40, "line"), (30, "full"), (64, "3D"), (100, "Imp3D"), (27, "3D"), (1, "3D")])
def test_topology_orders_match_program_fs(n, topo):
    o = Oracle(n, topo, "gossip", seed=5)
    P, _, g = srs_py.resolve(n, topo)
    nbrs, _ = srs_py.build_neighbours(P, g, topo, 5)
    assert len(nbrs) == o.P
    for i in range(o.P):
        assert o.neighbors(i) == nbrs[i], i


def test_imp3d_random_edge_range():
    # Random().Next(0, nodes-1) -> [0, P-2] (Program.fs:259); never points at P-1 (Q4)
    P, _, g = srs_py.resolve(1000, "Imp3D")
    o = Oracle(1000, "Imp3D", "gossip", seed=11)
    rnd = [o.neighbors(i)[-1] for i in range(P)]
    assert max(rnd) <= P - 2 and min(rnd) >= 0


def _digest(alg, st):
    h = hashlib.sha256()
    if alg == "gossip":
        h.update(st["c"].astype("<i4").tobytes())
    else:
        h.update(st["s"].astype("<f8").tobytes())
        h.update(st["w"].astype("<f8").tobytes())
    h.update(st["flags"].astype("u1").tobytes())
    return h.hexdigest()


def golden_cases():
    with open(GOLDEN) as f:
        return json.load(f)["cases"]


@pytest.mark.parametrize("case", golden_cases(), ids=lambda c: f"{c['topology']}-{c['algorithm']}-{c['num_nodes']}-s{c['seed']}")
def test_c_oracle_matches_golden(case):
    o = Oracle(case["num_nodes"], case["topology"], case["algorithm"], case["seed"])
    assert (o.P, o.T, o.seed_node) == (case["population"], case["threshold"], case["seed_node"])
    alerts = o.step(case["max_rounds"])
    assert alerts == case["alerts_per_round"]
    assert _digest(case["algorithm"], o.state()) == case["state_sha256"]


@pytest.mark.parametrize("n,topo,alg,seed", [(20, "line", "gossip", 4), (25, "full", "push-sum", 9),
                                             (27, "3D", "gossip", 6), (64, "Imp3D", "push-sum", 8),
                                             (125, "Imp3D", "gossip", 10)])
def test_c_oracle_vs_python_oracle(n, topo, alg, seed):
    o, p = Oracle(n, topo, alg, seed), srs_py.PySim(n, topo, alg, seed)
    assert o.step(2000) == p.step(2000)
    st = o.state()
    if alg == "gossip":
        assert list(st["c"]) == p.c
    else:
        assert list(st["s"]) == p.s and list(st["w"]) == p.w
    assert list(st["flags"]) == p.flags()


@pytest.mark.parametrize("topo", ["line", "full", "3D", "Imp3D"])
def test_pushsum_invariants(topo):
    """Mass conservation (sum s = P(P-1)/2, sum w = P) to 1e-12 relative; sticky convergence."""
    o = Oracle(4096, topo, "push-sum", seed=3)
    P = o.P
    prev_conv = np.zeros(P, bool)
    for _ in range(20):
        o.step(10)
        st = o.state()
        assert abs(st["s"].sum() - P * (P - 1) / 2) <= 1e-12 * P * (P - 1) / 2
        assert abs(st["w"].sum() - P) <= 1e-12 * P
        conv = (st["flags"] & 2) != 0
        assert np.all(conv[prev_conv])
        assert conv.sum() == o.alerts_total
        prev_conv = conv


@pytest.mark.parametrize("topo", ["line", "full", "3D", "Imp3D"])
def test_gossip_invariants(topo):
    """Counters monotone; each node alerts exactly once (alerts == #(c >= 11))."""
    o = Oracle(3000, topo, "gossip", seed=2)
    prev = np.zeros(o.P, np.int32)
    for _ in range(40):
        o.step(25)
        c = o.state()["c"]
        assert np.all(c >= prev)
        assert (c >= 11).sum() == o.alerts_total
        prev = c


@pytest.mark.parametrize("n,topo,seed,warms", [(27000, "Imp3D", 3, (3, 25, 150)), (64000, "Imp3D", 11, (3, 25, 150)),
                                                (8000, "3D", 5, (3, 25, 150)), (3000, "line", 2, (3, 25, 150)),
                                                (20000, "full", 4, (3, 20, 60, 108, 111, 116))])
def test_pushsum_receivers_matches_whole_network_round(n, topo, seed, warms):
    """or_pushsum_receivers (one round for sampled receivers, pulled from a full
    round-start state -- the checker of the P = 1e9 GPU round and of the full
    topology's alert phase at P = 1e8) equals the whole-network oracle's round, bit
    for bit, during activation, in steady state and (full) while nodes converge;
    its return value counts the sampled receivers that converge in the round."""
    from tests.oracle_ctypes import pushsum_receivers
    orc = Oracle(n, topo, "push-sum", seed)
    P = orc.P
    rng = np.random.default_rng(seed)
    for warm in warms:
        orc.step(warm - orc.rounds) if warm > orc.rounds else None
        st = orc.state()
        r = orc.rounds
        ids = np.unique(np.concatenate([rng.choice(P, size=min(P, 2000), replace=False),
                                        np.arange(min(P, 300)), np.arange(P - 300, P)]))
        so, wo, fo, conv = pushsum_receivers(topo, n, seed, r, st["s"], st["w"], st["flags"], ids)
        assert len(orc.step(1)) == 1
        nx = orc.state()
        np.testing.assert_array_equal(so, nx["s"][ids])
        np.testing.assert_array_equal(wo, nx["w"][ids])
        np.testing.assert_array_equal(fo, nx["flags"][ids])
        assert conv == int(np.count_nonzero((nx["flags"][ids] & 2) & ~(st["flags"][ids] & 2)))
    orc.close()


def test_activate_all_is_a_steady_state_round():
    """Oracle.activate_all (bench.py's CPU-baseline sample only): every node active, and
    a round after it sends from every node and conserves the mass, like any round."""
    from tests.oracle_ctypes import Oracle
    orc = Oracle(27000, "Imp3D", "push-sum", 1, threads=1)
    P = orc.P
    assert orc.activate_all() == P - 1  # the seed was already active
    assert orc.active_count() == P
    st0 = orc.state()
    orc.step(1)
    st1 = orc.state()
    assert abs(st1["s"].sum() - st0["s"].sum()) <= 1e-9 * abs(st0["s"].sum())
    assert abs(st1["w"].sum() - P) <= 1e-9 * P
    assert (st1["w"] != 1.0).sum() > P // 2  # every node halved and/or received
    orc.close()
    assert Oracle(1000, "line", "gossip", 1).activate_all() == -1
