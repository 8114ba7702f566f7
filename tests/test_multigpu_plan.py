"""CPU: the one-node 8-GPU plan of BASELINE's multi-GPU configurations, computed on
the host (no GPU, no RCCL).  The library's slab plan (gp_api.hip make_bounds)
and exchange capacities (gp_api.hip setup_exchange: expected messages per rank
pair + 12 sigma + 64) are restated here; the tests check that

  * C5 (Imp3D push-sum, n = 1e9) and C4 (full push-sum, n = 1e8) fit one
    MI355X's 288 GB per rank at world 8, setup temporaries included;
  * the fixed capacities leave a 12-sigma margin over the per-round message
    count, so an overflow (which fails the run loudly, tests/test_gpu_multirank)
    is not a practical event over a convergence run;
  * at a size the emulation can draw exactly (world 8, P = 64,000), the realised
    per-pair counts of every round stay below the capacities the formula gives.
"""
import math

import pytest

import numpy as np

from tests.multirank_emu import (DIR_RANDOM, Geometry, S_PUSHSUM, S_TOPO, full_bin_multi_cap, full_bin_multi_s1,
                                 full_region, resolve, slab_bounds, uniform)

HBM_BYTES = 288e9
GAUSS_12SIGMA_TAIL = 1.8e-33  # P(Z > 12)


def imp3d_pair_stats(P, g, W):
    """Expected random-edge messages per round for every rank pair a -> b and their
    variance, from the degree distribution of the lattice (rnd[i] uniform in
    [0, P-2], a sender uses its random edge with probability 1/deg)."""
    bounds, _ = slab_bounds(P, g, "Imp3D", W)
    # 1/deg summed over a slab's senders: interior 1/7, face 1/6, edge 1/5, corner 1/4
    def inv_deg_sum(x0, x1):
        tot = 0.0
        for x in (x0, x1 - 1) if x1 - x0 > 1 else (x0,):
            pass
        n_int_x = max(0, min(x1, g - 1) - max(x0, 1))  # planes with both x neighbours
        n_bnd_x = (x1 - x0) - n_int_x
        # per plane: g^2 nodes; y/z boundary counts
        inner = (g - 2) ** 2
        faces = 4 * (g - 2)
        corners = 4
        for planes, xb in ((n_int_x, 0), (n_bnd_x, 1)):
            # degree = 1 (random) + 6 lattice - boundary count
            tot += planes * (inner / (7 - xb) + faces / (6 - xb) + corners / (5 - xb))
        return tot
    mu = np.zeros((W, W))
    var = np.zeros((W, W))
    for a in range(W):
        x0, x1 = bounds[a] // (g * g), bounds[a + 1] // (g * g)
        s = inv_deg_sum(x0, x1)
        for b in range(W):
            if a == b:
                continue
            frac = (bounds[b + 1] - bounds[b]) / (P - 1)  # share of targets on rank b
            mu[a, b] = s * frac
            var[a, b] = mu[a, b] * (1 - 1 / 7)
    return bounds, mu, var


def cap_of(mu):
    return math.ceil(mu + 12.0 * math.sqrt(mu) + 64.0)


def imp3d_rank_bytes(nloc, halo, nedges, W, caps_out, caps_in, P):
    """Device bytes of one Imp3D push-sum rank (alloc_slab + build_imp3d + build_lists +
    setup_exchange), and the peak with build_imp3d's global temporaries.  Since round 5 the
    random-edge exchange is sender-ordered lists: per in-edge the list key rk (no slot, tag
    or message arrays), per sender its static list rank xdr (2 B), and per pair and region
    one 16-B header word per 64 list entries (about half a word of padding per tile) plus
    the message slots, on both sides."""
    next_ = nloc + 2 * halo + 1024
    node = next_ * (2 * 16 + 2) + nloc * 4 + (nloc + 5) * 4 + 2 * (nloc // 64 + 64) * 8  # sw, nb, rnd, in_off, rbits
    node += nloc * (1 + 2)                                                               # xdst, xdr
    edges = (nedges + 4) * 4 * 3                                                         # in_src, in_srcd, rk
    tiles = nloc // 1024 + 2
    hdr = 2 * 16 * (nedges / 64 + tiles * W / 2)                                         # header words, out and in
    xbuf = hdr + sum(16 * c for c in caps_out) + sum(16 * c for c in caps_in)
    steady = node + edges + xbuf
    temporaries = P * 4 * 7 + 64e6  # rnd_all, iota (then the list keys), keys, src_sorted, counts, off_all, inv + sort scratch
    return steady, steady + temporaries


def test_c5_imp3d_pushsum_1e9_world8_plan():
    P, T, g = resolve(10**9, "Imp3D")
    W = 8
    bounds, mu, var = imp3d_pair_stats(P, g, W)
    assert [(bounds[w + 1] - bounds[w]) // (g * g) for w in range(W)] == [125] * 8  # planes per rank
    for a in range(W):
        # push-sum: two regions per pair, one per half of the sender's slab, each sized for
        # its own expectation (setup_exchange; both halves hold ~half of the pair's senders)
        caps_out = [cap_of(mu[a, b] / 2) if b != a else 0 for b in range(W) for _ in range(2)]
        caps_in = [cap_of(mu[b, a] / 2) if b != a else 0 for b in range(W) for _ in range(2)]
        for b in range(W):
            if b == a:
                continue
            margin = (cap_of(mu[a, b] / 2) - mu[a, b] / 2) / math.sqrt(var[a, b] / 2)
            assert margin >= 12.0  # per-round overflow probability below GAUSS_12SIGMA_TAIL
            assert 2.0e6 < mu[a, b] < 2.5e6  # ~2.2 M messages per pair per round
        nloc = bounds[a + 1] - bounds[a]
        steady, peak = imp3d_rank_bytes(nloc, g * g, nloc, W, caps_out, caps_in, P)
        assert peak < 0.8 * HBM_BYTES, f"rank {a}: {peak / 1e9:.1f} GB"
        assert steady < 0.1 * HBM_BYTES
    # a convergence run of 10^5 rounds x 56 pairs stays far from an overflow
    assert 1e5 * W * (W - 1) * GAUSS_12SIGMA_TAIL < 1e-25


def full_bin_plan(nrecv, fused=False):
    """gp_fullbin.hip full_bin_plan: coarse bins of 2^s1 receivers, fine tiles of 4096; the
    fused fold (one rank) takes coarse bins one size smaller, at most 1024 of them."""
    fb_tb, cap2 = 12, 4992
    bits = 1
    while bits < 32 and (1 << bits) < nrecv:
        bits += 1
    s1 = max((bits + fb_tb + 1) // 2 - (1 if fused else 0), fb_tb)
    while (nrecv >> s1) >= 4096:
        s1 += 1
    while fused and ((nrecv + (1 << s1) - 1) >> s1) > 1024:
        s1 += 1
    while s1 - fb_tb > 12:
        s1 -= 1
    nb1 = (nrecv + (1 << s1) - 1) >> s1
    nb2 = (nrecv + (1 << fb_tb) - 1) >> fb_tb
    m1 = (1 << s1) * (nrecv / max(nrecv - 1, 1))
    return nb1, int(m1 + 12.0 * math.sqrt(m1) + 1024.0), nb2, cap2


def fb_bins_bytes(nb, cap):
    """gp_fullbin.hip fb_bins_bytes: [counts | sender ids | payloads], 16-B aligned parts."""
    return (nb * 4 + 15) // 16 * 16 + (nb * cap * 4 + 15) // 16 * 16 + nb * cap * 16


@pytest.mark.parametrize("W", [2, 4, 8])
def test_c4_full_pushsum_1e8_plan(W):
    """Several ranks (round 6, gp_fullbin.hip k_fb_fold<FOLD_SEND_RANKS>): the fold of each of a
    slab's two exchange regions (whole fine tiles) bins its nodes' next-round messages by
    destination rank and the destination's coarse bin -- 2^s1 receivers, one size on every rank
    -- into fixed-capacity bins that travel as the exchange buffers (own share into the rank's
    own receive region), and the receiver's split reads them where they arrive.  The capacity
    per (region, pair, bin) is Binomial(n_region, 2^s1 / (P - 1)) + 12 sigma + 64."""
    P, T, _ = resolve(10**8, "full")
    bounds, halo = slab_bounds(P, 0, "full", W)
    assert halo == 0 and bounds[-1] == P
    s1 = full_bin_multi_s1(bounds)
    nb = [-(-(bounds[b + 1] - bounds[b]) // (1 << s1)) for b in range(W)]
    assert s1 == 19 and sum(nb) <= 192  # within the fold's LDS keys (1024), runs of ~21 per (tile, key)
    q = (1 << s1) / (P - 1)
    for a in range(W):
        na = bounds[a + 1] - bounds[a]
        out_bytes = in_bytes = 0
        for h in range(2):
            r0, r1 = full_region(na, 2, h)
            cap = full_bin_multi_cap(r1 - r0, s1, P)
            m = (r1 - r0) * q
            assert (cap - m) / math.sqrt(m * (1 - q)) >= 12.0
            assert cap / m - 1 < 0.08  # the fixed capacities' share of the wire bytes
            out_bytes += sum(fb_bins_bytes(nb[b], cap) for b in range(W) if b != a)
            for p in range(W):
                n_p = bounds[p + 1] - bounds[p]
                p0, p1 = full_region(n_p, 2, h)
                in_bytes += fb_bins_bytes(nb[a], full_bin_multi_cap(p1 - p0, s1, P))
        # the messages a sends per round: 20 B each; the buffers add under 8 %
        msgs = na * (P - na) / (P - 1) * 20
        assert out_bytes < 1.08 * msgs + 1e6
        nb2, cap2 = -(-na // 4096), 4992
        steady = na * (2 * 16 + 1) + out_bytes + in_bytes + nb2 * cap2 * 20
        assert steady < 0.5 * HBM_BYTES


def test_realised_imp3d_counts_stay_below_capacity_world8():
    """Exact per-round counts at P = 64,000 (g = 40, 5 planes per rank), every
    node active: the messages each rank pair carries in 40 rounds, drawn from
    the same Philox streams as the library, against the capacity formula fed
    with the realised expectation (as setup_exchange computes it)."""
    n, W, seed = 64000, 8, 5
    P, T, g = resolve(n, "Imp3D")
    geo = Geometry(P, g, "Imp3D", seed)
    bounds, _ = slab_bounds(P, g, "Imp3D", W)
    ids = np.arange(P)
    rnd = uniform(seed, S_TOPO, ids, 0, P - 1)
    src_rank = np.searchsorted(np.array(bounds[1:-1]), ids, side="right")
    dst_rank = np.searchsorted(np.array(bounds[1:-1]), rnd, side="right")
    inv_deg = 1.0 / geo.degree(ids)
    # push-sum exchange region of every sender (setup_exchange / build_lists): its tile's quarter
    # of the slab's 1024-id tiles (tiles on global multiples of 1024; region h: tiles
    # [nt h / NH, nt (h + 1) / NH), NH = 4)
    NH = 4
    b_arr = np.array(bounds)
    lo_t = b_arr[src_rank] // 1024
    nt = (b_arr[src_rank + 1] + 1023) // 1024 - lo_t
    t_rel = ids // 1024 - lo_t
    half = np.zeros(P, dtype=np.int64)
    for h in range(1, NH):
        half += (t_rel >= nt * h // NH).astype(np.int64)
    mu = np.zeros((NH, W, W))
    np.add.at(mu, (half, src_rank, dst_rank), inv_deg)
    cap = np.vectorize(lambda m: min(cap_of(m), 10**9))(mu)
    worst = 0.0
    off = np.broadcast_to(~np.eye(W, dtype=bool), (NH, W, W))
    for r in range(40):
        d = geo.draw_dir(ids, S_PUSHSUM, r)
        sent = d == DIR_RANDOM
        cnt = np.zeros((NH, W, W), dtype=np.int64)
        np.add.at(cnt, (half[sent], src_rank[sent], dst_rank[sent]), 1)
        assert np.all(cnt[off] <= cap[off])
        worst = max(worst, float(np.max((cnt[off] - mu[off]) / np.sqrt(mu[off]))))
    assert worst < 6.0  # realised fluctuations are a few sigma; the capacity allows 12


@pytest.mark.parametrize("P", [2, 4097, 10**6, 100000001, 2**31 + 5, 2**32 - 1])
def test_fused_full_bin_plan_fits(P):
    """One rank runs the fused fold (k_fb_fold<true>) whenever its coarse bins fit the fold's
    1024 LDS reservation slots: the plan keeps every population up to 2^32 - 1 inside that,
    the fine tiles of a coarse bin within the split's 4096 LDS counters, and the bins' total
    capacity above the population (the 12-sigma slack of gp_fullbin.hip)."""
    nb1, cap1, nb2, cap2 = full_bin_plan(P, fused=True)
    assert nb1 <= 1024
    assert nb1 * cap1 >= P and nb2 * cap2 >= P
    nb1_rule = full_bin_plan(P)[0]
    assert nb1 >= nb1_rule  # one size smaller bins (more of them), unless the 1024 cap binds
    if P == 100000001:
        assert (nb1, nb1_rule) == (191, 96)


def halo_chunk_cap(g, imp3d):
    """gp_xchg.hip halo_chunk_cap: the senders toward one x neighbour in a 1024-node chunk of a
    slab-boundary plane are a sum of Bernoulli(1 / deg); the largest mean + 12 sigma over the
    plane's chunks, rounded up to 8."""
    y, z = np.divmod(np.arange(g * g), g)
    deg = 2 + (y > 0) + (y < g - 1) + (z > 0) + (z < g - 1) + (1 if imp3d else 0)
    p = 1.0 / deg
    best = 0.0
    for c0 in range(0, g * g, 1024):
        q = p[c0:c0 + 1024]
        best = max(best, q.sum() + 12.0 * math.sqrt((q * (1 - q)).sum()))
    return min(1024, max(8, (math.ceil(best) + 7) // 8 * 8)), p


def poisson_binomial_tail(q, k):
    """P(sum of Bernoulli(q_i) > k), exactly (dynamic programme over the chunk's nodes)."""
    dist = np.zeros(len(q) + 2)
    dist[0] = 1.0
    for n, qi in enumerate(q):
        dist[1:n + 2] = dist[1:n + 2] * (1 - qi) + dist[0:n + 1] * qi
        dist[0] *= 1 - qi
    return float(dist[k + 1:].sum())


@pytest.mark.parametrize("g,imp3d", [(1000, False), (1000, True), (465, True), (100, False), (1625, False)])
def test_halo_chunk_capacity_covers_boundary_rows(g, imp3d):
    """A chunk made of a plane's boundary row (y = 0: degree 5 on 3D, 6 on Imp3D) sends toward
    x -+ 1 with probability 1/5 (1/6), not the interior 1/7: round 5's fixed 256 slots overflowed
    with probability ~3e-5 per chunk and round on 3D at g = 1000 (a loud but spurious GP_ESTATE).
    The capacity rule keeps every chunk's exact overflow probability negligible over a
    convergence run (every round, both directions, every slab boundary)."""
    cap, p = halo_chunk_cap(g, imp3d)
    worst = max(poisson_binomial_tail(p[c0:c0 + 1024], cap) for c0 in (0, 1024, (g * g // 1024) * 1024 - 1024))
    assert worst < 1e-25
    if g == 1000:
        assert cap == (360 if not imp3d else 320)
        row0 = p[0:1024]
        if not imp3d:
            assert 3e-5 < poisson_binomial_tail(row0, 256) < 4e-5  # the round-5 capacity
