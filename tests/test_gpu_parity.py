"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle.

Bar (north star): gossip counters and convergence round bit-exact; push-sum
s/w -- also bit-exact here (the kernels fold in the oracle's canonical order
with -ffp-contract=off; the north star's 1e-12 relative tolerance is the
fallback and is what the size-independent checks below use).
"""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

from tests.oracle_ctypes import Oracle

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "srs_v1_golden.json")


def Sim(*a, **k):
    from gossipprotocol_amd import Simulation
    return Simulation(*a, **k)


def digest(alg, st):
    h = hashlib.sha256()
    if alg == "gossip":
        h.update(st["c"].astype("<i4").tobytes())
    else:
        h.update(st["s"].astype("<f8").tobytes())
        h.update(st["w"].astype("<f8").tobytes())
    h.update(st["flags"].astype("u1").tobytes())
    return h.hexdigest()


def assert_same_state(alg, gs, os_):
    if alg == "gossip":
        np.testing.assert_array_equal(gs["c"], os_["c"])
    else:
        np.testing.assert_array_equal(gs["s"], os_["s"])
        np.testing.assert_array_equal(gs["w"], os_["w"])
    np.testing.assert_array_equal(gs["flags"], os_["flags"])


with open(GOLDEN) as _f:
    GOLDEN_CASES = json.load(_f)["cases"]


@pytest.mark.parametrize("case", GOLDEN_CASES,
                         ids=lambda c: f"{c['topology']}-{c['algorithm']}-{c['num_nodes']}-s{c['seed']}")
def test_golden(case):
    sim = Sim(case["num_nodes"], case["topology"], case["algorithm"], seed=case["seed"])
    assert (sim.population, sim.threshold, sim.seed_node) == (case["population"], case["threshold"],
                                                              case["seed_node"])
    alerts = sim.step(case["max_rounds"])
    assert alerts == case["alerts_per_round"]
    assert sim.rounds == case["rounds"]
    assert digest(case["algorithm"], sim.state()) == case["state_sha256"]
    sim.close()


LIVE = [  # (num_nodes, topology, algorithm, seed, rounds, checkpoint)
    (64000, "Imp3D", "push-sum", 5, 600, 97),
    (125000, "Imp3D", "gossip", 7, 400, 101),
    (216000, "3D", "push-sum", 9, 300, 150),
    (8000, "3D", "gossip", 4, 3000, 1000),
    (5000, "line", "gossip", 6, 8000, 2000),
    (777, "line", "push-sum", 2, 2000, 500),
    (50000, "full", "gossip", 3, 400, 100),
    (30000, "full", "push-sum", 8, 300, 50),
]


@pytest.mark.parametrize("n,topo,alg,seed,rounds,chk", LIVE, ids=lambda v: str(v))
def test_live_parity(n, topo, alg, seed, rounds, chk):
    """Bit-exact state at several checkpoints, per-round alerts identical."""
    sim, orc = Sim(n, topo, alg, seed=seed), Oracle(n, topo, alg, seed)
    done = 0
    while done < rounds:
        k = min(chk, rounds - done)
        ga, oa = sim.step(k), orc.step(k)
        assert ga == oa, f"alerts differ in rounds {done}..{done + k}"
        assert_same_state(alg, sim.state(), orc.state())
        done += k
        if len(ga) < k:
            break
    assert sim.rounds == orc.rounds and sim.alerts_total == orc.alerts_total
    sim.close()


@pytest.mark.parametrize("n", [1, 2, 3, 1023, 1024, 4095, 4096, 16383, 16384, 65535, 65536, 131071])
def test_full_pushsum_boundary_sizes(n):
    """Full push-sum (range binning, gp_fullbin.hip) at populations P = n + 1 on and
    around its chunk (4096 messages), work-item (16384 senders) and fine-tile (4096
    receivers) sizes: bit-exact state every 25 rounds through convergence.  One rank
    runs the fused form: round 0's send pass, then every fold bins the next round's
    messages (k_fb_fold<true>)."""
    sim, orc = Sim(n, "full", "push-sum", seed=n + 3), Oracle(n, "full", "push-sum", n + 3)
    assert sim.kernel_stats()[2] == "k_fb_split+fold<send>"
    done = 0
    while done < 400:
        ga, oa = sim.step(25), orc.step(25)
        assert ga == oa, f"alerts differ in rounds {done}..{done + 25}"
        assert_same_state("push-sum", sim.state(), orc.state())
        done += 25
        if len(ga) < 25:
            break
    assert sim.rounds == orc.rounds and sim.alerts_total == orc.alerts_total
    sim.close()


@pytest.mark.parametrize("n,seed", [(4095, 11), (131071, 12), (2000000, 13)])
def test_full_pushsum_three_pass_parity(n, seed, monkeypatch):
    """The three-pass full push-sum round (send, split, fold every round; experiments
    build, GP_FB_FUSED=0) stays bit-exact too: it is the form several ranks run
    (k_fbm_send bins by destination rank), and the A/B reference for the fused one."""
    monkeypatch.setenv("GP_FB_FUSED", "0")
    sim, orc = Sim(n, "full", "push-sum", seed=seed, experimental=True), Oracle(n, "full", "push-sum", seed)
    assert sim.kernel_stats()[2] == "k_fb_send+split+fold"
    for _ in range(4):
        ga, oa = sim.step(30), orc.step(30)
        assert ga == oa
        assert_same_state("push-sum", sim.state(), orc.state())
        if len(ga) < 30:
            break
    sim.close()


def test_step_chunking_is_invisible():
    a = Sim(27000, "Imp3D", "push-sum", seed=12)
    b = Sim(27000, "Imp3D", "push-sum", seed=12)
    alerts_a = a.step(2000)
    alerts_b = []
    for k in (1, 2, 3, 5, 7, 11, 64, 100, 333, 1024, 2000):
        alerts_b += b.step(k)
    assert alerts_a == alerts_b[: len(alerts_a)] and a.rounds == b.rounds
    assert digest("push-sum", a.state()) == digest("push-sum", b.state())


@pytest.mark.parametrize("n,topo", [(50, "line"), (40, "full"), (1000, "3D"), (1000, "Imp3D")])
def test_neighbors_match_oracle(n, topo):
    sim, orc = Sim(n, topo, "gossip", seed=21), Oracle(n, topo, "gossip", 21)
    for i in list(range(0, orc.P, max(1, orc.P // 97))) + [orc.P - 1]:
        assert sim.neighbors(i) == orc.neighbors(i)


def test_max_rounds_cap():
    sim = Sim(1000, "line", "push-sum", seed=1, max_rounds=123)
    res = sim.run()
    assert res.status == 1 and res.rounds == 123


def test_cli_contract():
    exe = os.path.join(ROOT, "gossipprotocol_amd", "gossip")
    r = subprocess.run([exe, "1000", "line", "gossip"], capture_output=True, text=True, timeout=120)
    lines = r.stdout.splitlines()
    assert r.returncode == 0, r.stderr
    assert lines[0] == "Gossip Starts" and lines[1].startswith("Convergence Time: ") and lines[1].endswith(" ms")
    r = subprocess.run([exe, "1000", "imp3D", "push-sum"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.splitlines()[0] == "Push Sum Starts"


def test_large_imp3d_pushsum_parity_1e8():
    """BASELINE config sizes: g = 465 (P = 100,544,625), first rounds bit-exact vs the oracle."""
    n, rounds = 10**8, 6
    sim, orc = Sim(n, "Imp3D", "push-sum", seed=1), Oracle(n, "Imp3D", "push-sum", 1)
    assert sim.step(rounds) == orc.step(rounds)
    gs, os_ = sim.state(), orc.state()
    assert_same_state("push-sum", gs, os_)
    sim.close()
    orc.close()


def _read_all(sim, P, chunk=50_000_000):
    """Full push-sum state of a P-node simulation: s, w, flags (chunked readback)."""
    s = np.empty(P, np.float64)
    w = np.empty(P, np.float64)
    f = np.empty(P, np.uint8)
    for first in range(0, P, chunk):
        cnt = min(chunk, P - first)
        st = sim.state(first, cnt)
        s[first:first + cnt] = st["s"]
        w[first:first + cnt] = st["w"]
        f[first:first + cnt] = st["flags"]
    return s, w, f


def _sample_ids(P, g, rng, n_random=1_000_000):
    """Receivers checked at P = 1e9: 1e6 uniform ones plus every node of whole
    blocks where the kernels' data layout has edges -- the planes x = 0 and g - 1
    (rows y < 40), patch boundary rows (y = 7, 8, 15, 16, 991, 992, ...), z-segment
    boundaries (z = 63, 64, 959, 960, 999) on every 25th plane, the last row."""
    g2 = g * g
    ids = [rng.choice(P, size=n_random, replace=False)]
    rows = np.arange(40)
    for x in (0, g - 1):
        ids.append((x * g2 + (rows[:, None] * g + np.arange(g)[None, :])).ravel())
    ys = np.array([7, 8, 15, 16, 31, 32, g // 2, g - 9, g - 8, g - 1])
    zs = np.array([0, 1, 62, 63, 64, 65, 959, 960, g - 2, g - 1])
    xs = np.arange(0, g, 25)
    ids.append((xs[:, None, None] * g2 + ys[None, :, None] * g + np.arange(g)[None, None, :]).ravel())
    ids.append((xs[:, None, None] * g2 + np.arange(g)[None, :, None] * g + zs[None, None, :]).ravel())
    return np.unique(np.concatenate(ids).astype(np.int64))


def _check_round_sampled(sim, n, seed, ids, topology="Imp3D"):
    """Round r of the GPU (r = sim.rounds) against or_pushsum_receivers for ids.
    Also: the round's alert count reported by the GPU equals the number of nodes
    whose converged flag the round set (whole state), and the sampled receivers
    that converge in it are exactly the ones the oracle says converge."""
    from tests.oracle_ctypes import pushsum_receivers
    P = sim.population
    r = sim.rounds
    s, w, f = _read_all(sim, P)
    tot = (float(np.sum(s)), float(np.sum(w)))
    so, wo, fo, conv_sampled = pushsum_receivers(topology, n, seed, r, s, w, f, ids)
    conv0 = int(np.count_nonzero(f & 2))
    was_conv = (f[ids] & 2) != 0
    del s, w, f
    alerts = sim.step(1)
    assert sim.rounds == r + 1 and len(alerts) == 1
    s2, w2, f2 = _read_all(sim, P)
    np.testing.assert_array_equal(s2[ids], so, err_msg=f"s differs in round {r}")
    np.testing.assert_array_equal(w2[ids], wo, err_msg=f"w differs in round {r}")
    np.testing.assert_array_equal(f2[ids], fo, err_msg=f"flags differ in round {r}")
    newly = int(np.count_nonzero(((f2[ids] & 2) != 0) & ~was_conv))
    assert newly == conv_sampled, f"round {r}: {newly} sampled receivers converged, oracle says {conv_sampled}"
    assert alerts[0] == int(np.count_nonzero(f2 & 2)) - conv0, f"round {r}: alert count != newly converged nodes"
    return tot, alerts[0], conv_sampled


class _C5:
    """The one P = 1e9 run the full-size tests below share (module fixture), so each
    segment reports as it finishes."""
    n, seed = 10**9, 1


@pytest.fixture(scope="module")
def c5():
    st = _C5()
    st.sim = Sim(st.n, "Imp3D", "push-sum", seed=st.seed)
    st.P, g = st.sim.population, st.sim.info().grid
    st.ids = _sample_ids(st.P, g, np.random.default_rng(7))
    st.ref_s = st.P * (st.P - 1) / 2
    st.hash41 = None
    yield st
    st.sim.close()


def _c5_check(st):
    (tot_s, tot_w), a, conv = _check_round_sampled(st.sim, st.n, st.seed, st.ids)
    assert abs(tot_s - st.ref_s) <= 1e-12 * st.ref_s  # mass conserved
    assert abs(tot_w - st.P) <= 1e-12 * st.P
    return a, conv


# C5 at its real size (P = 1e9), on the kernel bench.py times: rounds recomputed on
# the host for ~1.1e6 receivers by or_pushsum_receivers from the read-back
# round-start state -- bit-exact s, w and flags (Program.fs:101-131 via SRS v1
# B.4) -- during activation (round 40), in steady state before any alert (every
# node active, 8 rounds later), at the alert peak (round 533: 1.5e7 of the 1e9
# nodes converge in that round, the count / converge branch of Program.fs:114-123)
# and in the tail (round 700: 99 % converged, converged nodes forwarding, D6); mass
# conserved to 1e-12 relative; each round's alert count equals the nodes it
# converged; a second run is bit-identical (determinism).
def test_full_size_1e9_activation_round(c5):
    c5.sim.step(40)
    _c5_check(c5)
    c5.hash41 = hashlib.sha256(c5.sim.state(0, 50_000_000)["s"].tobytes()).hexdigest()


def test_full_size_1e9_steady_round(c5):
    assert c5.sim.rounds == 41
    while c5.sim.info().active < c5.P:
        assert c5.sim.rounds < 400, "activation did not complete"
        c5.sim.step(8)
    c5.sim.step(8)
    assert c5.sim.info().active == c5.P
    _c5_check(c5)


def test_full_size_1e9_alert_peak_round(c5):
    c5.sim.step(533 - c5.sim.rounds)
    a, conv = _c5_check(c5)
    assert a > 10**7 and conv > 5000, (a, conv)  # the alert peak is exercised


def test_full_size_1e9_tail_round(c5):
    c5.sim.step(700 - c5.sim.rounds)
    a, conv = _c5_check(c5)
    assert a > 10**5 and c5.sim.alerts_total > 0.98 * c5.P, (a, c5.sim.alerts_total)


def test_full_size_1e9_determinism(c5):
    assert c5.hash41 is not None
    c5.sim.close()
    sim2 = Sim(c5.n, "Imp3D", "push-sum", seed=c5.seed)
    sim2.step(41)
    assert hashlib.sha256(sim2.state(0, 50_000_000)["s"].tobytes()).hexdigest() == c5.hash41
    sim2.close()


def test_full_pushsum_1e8_alert_phase_sampled():
    """C4 (full push-sum, P = 100,000,001) in its alert phase: the round in which the
    cumulative alerts first pass 10 % of T and the one in which they pass 99 % are
    recomputed on the host for ~1e6 sampled receivers (or_pushsum_receivers, full
    topology: every active sender's Philox target, folded by ascending sender id,
    Program.fs:209-216,101-131) -- bit-exact s, w, flags; the round's alert count
    equals the nodes it converged; mass conserved.  (The whole-network comparison
    through convergence is tests/test_gpu_baseline_sizes.py's C4 run.)"""
    n, seed = 10**8, 1
    sim = Sim(n, "full", "push-sum", seed=seed)
    P, T = sim.population, sim.threshold
    rng = np.random.default_rng(5)
    ids = np.unique(np.concatenate([rng.choice(P, size=1_000_000, replace=False), np.arange(2000),
                                    np.arange(P - 2000, P)]).astype(np.int64))
    ref_s = P * (P - 1) / 2
    checked = []
    for frac in (0.10, 0.99):
        while sim.alerts_total < frac * T:
            assert sim.rounds < 2000 and len(sim.step(1)) == 1
        (tot_s, tot_w), a, conv = _check_round_sampled(sim, n, seed, ids, topology="full")
        assert abs(tot_s - ref_s) <= 1e-12 * ref_s and abs(tot_w - P) <= 1e-12 * P
        checked.append((sim.rounds - 1, a, conv))
    assert all(a > 0 for _, a, _ in checked), checked
    sim.close()


KERNEL_CASES = [  # (num_nodes, topology, algorithm, seed, rounds, checkpoint, x-segments)
    (64000, "Imp3D", "push-sum", 5, 400, 97, "3"),
    (125000, "Imp3D", "gossip", 7, 300, 101, "2"),
    (216000, "3D", "push-sum", 9, 200, 75, "1"),
    (27000, "3D", "gossip", 4, 600, 150, "4"),
    (343000, "Imp3D", "push-sum", 11, 120, 60, "1"),
]


@pytest.mark.parametrize("kernel", ["col", "tile", "tile4", "tile1"])
@pytest.mark.parametrize("n,topo,alg,seed,rounds,chk,xsegs", KERNEL_CASES, ids=lambda v: str(v))
def test_kernel_variant_parity(kernel, n, topo, alg, seed, rounds, chk, xsegs, monkeypatch):
    """Every round-kernel variant (column march / tiled; experiments build,
    GP_KERNEL) bit-exact vs the oracle, the column march also with its
    x-segmentation forced; the tiled kernel in the size class its population
    selects (tile), forced to 256 threads x 4 nodes (tile4, GP_WIDE=0) and to the
    1024-thread x 1 node build (tile1, GP_WIDE=1, gp_round_wide.hip)."""
    if kernel == "col" and alg == "push-sum":
        pytest.skip("the column march runs lattice gossip only")
    if kernel == "tile1" and (alg != "push-sum" or topo == "Imp3D"):
        # GP_WIDE only selects among the line / 3D push-sum size classes (choose_kernel)
        pytest.skip("the 1024-thread build runs line / 3D push-sum only")
    monkeypatch.setenv("GP_KERNEL", "tile" if kernel.startswith("tile") else kernel)
    if kernel in ("tile4", "tile1"):
        monkeypatch.setenv("GP_WIDE", "1" if kernel == "tile1" else "0")
    monkeypatch.setenv("GP_XSEGS", xsegs)
    sim, orc = Sim(n, topo, alg, seed=seed, experimental=True), Oracle(n, topo, alg, seed)
    name = sim.kernel_stats()[2]
    if kernel in ("tile4", "tile1"):  # the size class the case claims to cover really runs
        assert name.startswith("wide::") == (kernel == "tile1"), name
    done = 0
    while done < rounds:
        k = min(chk, rounds - done)
        ga, oa = sim.step(k), orc.step(k)
        assert ga == oa, f"alerts differ in rounds {done}..{done + k}"
        assert_same_state(alg, sim.state(), orc.state())
        done += k
        if len(ga) < k:
            break
    sim.close()


WALK_CASES = [  # (num_nodes, topology, seed, rounds, checkpoint)
    (512000, "Imp3D", 3, 90, 45),
    (125000, "3D", 5, 120, 60),
]


@pytest.mark.parametrize("pack", ["0", "1"])
@pytest.mark.parametrize("walk", ["0", "1", "2"])
@pytest.mark.parametrize("n,topo,seed,rounds,chk", WALK_CASES, ids=lambda v: str(v))
def test_tile_walk_and_sender_packing_parity(n, topo, seed, rounds, chk, walk, pack, monkeypatch):
    """Push-sum tile kernel bit-exact vs the oracle for every tile walk (XCD eighths,
    global sweep, x-windows of 3 planes), with the senders' degree packed into the
    staged ids or computed (the P > 2^30 path); experiments build."""
    if topo != "Imp3D" and pack == "0":
        pytest.skip("sender packing is Imp3D only")
    monkeypatch.setenv("GP_KERNEL", "tile")
    monkeypatch.setenv("GP_WIDE", "0")  # the 256 x 4 kernel (the 1e9 one); its walks
    monkeypatch.setenv("GP_WALK", walk)
    monkeypatch.setenv("GP_WX", "3")
    monkeypatch.setenv("GP_NO_PACK", "0" if pack == "1" else "1")
    sim, orc = Sim(n, topo, "push-sum", seed=seed, experimental=True), Oracle(n, topo, "push-sum", seed)
    done = 0
    while done < rounds:
        k = min(chk, rounds - done)
        ga, oa = sim.step(k), orc.step(k)
        assert ga == oa, f"alerts differ in rounds {done}..{done + k}"
        assert_same_state("push-sum", sim.state(), orc.state())
        done += k
    if topo == "Imp3D":  # the steady-state (all nodes active) in-edge pass ran
        assert sim.info().active == sim.population
    sim.close()


@pytest.mark.parametrize("wide_at", ["2", "4"])
def test_nibble_wide_tile_fallback_parity(wide_at, monkeypatch):
    """Push-sum tile kernel: a tile holding a node whose in-degree does not fit the
    nibble array (>= 15, ~1e-12 of nodes, so never met by chance) reads in_off from
    HBM for all its nodes.  GP_IND4_WIDE (experiments build) lowers that mark so
    most (2) or some (4) tiles take the path; bit-exact vs the oracle through
    activation into steady state."""
    monkeypatch.setenv("GP_IND4_WIDE", wide_at)
    monkeypatch.setenv("GP_WIDE", "0")
    n, topo = 512000, "Imp3D"
    sim, orc = Sim(n, topo, "push-sum", seed=7, experimental=True), Oracle(n, topo, "push-sum", 7)
    for _ in range(2):
        ga, oa = sim.step(45), orc.step(45)
        assert ga == oa
        assert_same_state("push-sum", sim.state(), orc.state())
    assert sim.info().active == sim.population
    sim.close()


@pytest.mark.parametrize("kernel", ["col", "tile"])
def test_seed_random_edge_round0(kernel, monkeypatch):
    """Many seeds, so that several seed nodes send their round-0 rumour on the random
    edge: the column kernel's round-0 delivery count (k_col_seed_init) / the tile
    kernel's round-0 random-edge bitmap (k_rbits_init) must carry that send.
    Regression: the column layout's bitmap init once raced its own zeroing loop
    against the seed's bit (lost about one time in four)."""
    monkeypatch.setenv("GP_KERNEL", kernel)
    for seed in range(1, 25):
        sim, orc = Sim(27000, "Imp3D", "gossip", seed=seed, experimental=True), Oracle(27000, "Imp3D", "gossip", seed)
        assert sim.step(12) == orc.step(12), f"seed {seed}: alerts differ"
        assert np.array_equal(sim.state()["c"], orc.state()["c"]), f"seed {seed}: counters differ"
        sim.close()
        orc.close()


@pytest.mark.parametrize("wide", ["0", "1"])
@pytest.mark.parametrize("cap", ["0", "1000", "1024"])
def test_tile_unstaged_path_parity(cap, wide, monkeypatch):
    """Push-sum Imp3D tile kernel with the staging cap lowered (GP_STAGE_CAP): tiles
    with more in-edges than the cap take the unstaged path (per-edge decisions and
    gathers from HBM) -- all of them at 0, a mix at 1000 / 1024 (mean in-degree
    1024 per tile).  At the default cap (1216) that path runs for ~1e-9 of tiles."""
    if wide == "1":
        # the Imp3D push-sum kernel has one size class (its in-edge pass spills at 8 waves);
        # GP_WIDE does not reach it (choose_kernel), so wide=1 would repeat wide=0
        pytest.skip("Imp3D push-sum runs the 256 x 4 build only")
    monkeypatch.setenv("GP_KERNEL", "tile")
    monkeypatch.setenv("GP_WIDE", wide)
    monkeypatch.setenv("GP_STAGE_CAP", cap)
    n, seed, rounds, chk = 512000, 4, 90, 45
    sim, orc = Sim(n, "Imp3D", "push-sum", seed=seed, experimental=True), Oracle(n, "Imp3D", "push-sum", seed)
    done = 0
    while done < rounds:
        k = min(chk, rounds - done)
        ga, oa = sim.step(k), orc.step(k)
        assert ga == oa, f"alerts differ in rounds {done}..{done + k}"
        assert_same_state("push-sum", sim.state(), orc.state())
        done += k
    sim.close()


CLOSE_CASES = [  # (num_nodes, topology, seed, rounds, checkpoint): push-sum, one rank
    (2000000, "3D", 3, 120, 60),      # ~2000 blocks: uneven shard sizes (blockIdx % 8)
    (343000, "Imp3D", 6, 300, 100),
    (5000, "line", 8, 2000, 1000),    # one tile, a grid of 8 blocks (one per shard)
]


@pytest.mark.parametrize("n,topo,seed,rounds,chk", CLOSE_CASES, ids=lambda v: str(v))
@pytest.mark.parametrize("fuse", ["0", "1", "2"])
def test_round_close_parity(fuse, n, topo, seed, rounds, chk, monkeypatch):
    """Single-rank lattice push-sum closes its rounds three ways (experiments build,
    GP_FUSE): 0 a separate k_finalize launch, 1 the round kernel's last block via
    one arrival counter, 2 (product default) arrivals sharded over 8 counters whose
    last blocks forward to the global one.  Per-round alerts and full state
    bit-exact vs the oracle at every checkpoint, through convergence for line.
    GP_CHECK_CLOSE recounts the alerted nodes from the state after every batch and
    fails the step if the closes' bookkeeping disagrees."""
    monkeypatch.setenv("GP_FUSE", fuse)
    monkeypatch.setenv("GP_CHECK_CLOSE", "1")
    sim, orc = Sim(n, topo, "push-sum", seed=seed, experimental=True), Oracle(n, topo, "push-sum", seed)
    done = 0
    while done < rounds and orc.alerts_total < orc.T:
        k = min(chk, rounds - done)
        ga, oa = sim.step(k), orc.step(k)
        assert ga == oa, f"alerts differ in rounds {done}..{done + k}"
        assert_same_state("push-sum", sim.state(), orc.state())
        done += k
    assert sim.rounds == orc.rounds
    sim.close()
    orc.close()


BLOCK_CASES = [  # (num_nodes, seed, rounds, checkpoint): 3D push-sum, the LDS-resident kernel
    (1000, 3, 3000, 1000),        # one box, no grid barrier; through convergence
    (27000, 5, 400, 100),         # several boxes
    (8000, 7, 40000, 997),        # two boxes through convergence: batches and the converging
                                  # round cut epochs (16 rounds) mid-way -> checkpoint replay
    (1000000, 1, 300, 150),       # C2 (g = 100): one box per CU
    (1030301, 2, 120, 60),        # g = 101: uneven boxes
]


@pytest.mark.parametrize("n,seed,rounds,chk", BLOCK_CASES, ids=lambda v: str(v))
def test_block_kernel_parity(n, seed, rounds, chk, monkeypatch):
    """3D push-sum on the LDS-resident kernel (gp_block.hip: one cooperative launch per batch,
    boxes in LDS, faces through global memory at a grid barrier), forced with GP_KERNEL=block
    (experiments build): per-round alerts and full state bit-exact vs the oracle at every
    checkpoint (Program.fs:101-131, 238-257 via SRS v1 B.4), batches cut mid-run."""
    monkeypatch.setenv("GP_KERNEL", "block")
    sim, orc = Sim(n, "3D", "push-sum", seed=seed, experimental=True), Oracle(n, "3D", "push-sum", seed)
    assert sim.kernel_stats()[2] == "k_ps_block<GRID3D>"
    done = 0
    while done < rounds and orc.alerts_total < orc.T:
        k = min(chk, rounds - done)
        ga, oa = sim.step(k), orc.step(k)
        assert ga == oa, f"alerts differ in rounds {done}..{done + k}"
        assert_same_state("push-sum", sim.state(), orc.state())
        done += k
    assert sim.rounds == orc.rounds
    sim.close()
    orc.close()


def test_block_kernel_is_the_c2_default():
    """The product picks the LDS-resident kernel for C2 (3D push-sum, n = 1e6, one GPU)."""
    sim = Sim(10**6, "3D", "push-sum", seed=1)
    assert sim.kernel_stats()[2] == "k_ps_block<GRID3D>"
    sim.close()
