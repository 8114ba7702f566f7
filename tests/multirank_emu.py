"""CPU emulation of the multi-rank exchange protocol of libgossip_hip.so.

TEST INFRASTRUCTURE ONLY (tests/test_multirank_gloo.py).  Each torch.distributed
(gloo) rank owns the slab of node ids the library would give it
(gp_api.hip make_bounds: whole x-planes for 3D / Imp3D, contiguous ids for
line) and runs SRS v1 rounds for its slab with numpy, talking to the other
ranks only through the library's exchange plan:

  * halo refresh: after every round the boundary plane (line: node) of node
    bytes -- here the direction / active fields -- and (s, w) goes to the
    neighbouring rank (gp_api.hip exchange, halo part);
  * random-edge messages: every sender whose next direction is its random edge
    and whose target lives on another rank sends.  Push-sum: sender-ordered lists
    (ListPlan; gp_xchg.hpp k_list_pack) -- per region and destination one header
    word {bitmap, base} per 64 entries of the static list and the used entries'
    (s, w) compacted in list order; the receiver finds a remote in-edge's message
    from its list key (64 * header word + bit, build_lists) as base + the used
    entries below it.  Gossip (the column kernel's counts mode) {target's local
    id}, a rumour the receiver counts for the next round -- local senders count
    theirs at the target directly (k_gossip_col);
  * bookkeeping: {alerts, newly active, injector pick converged} summed over
    ranks (k_finalize_pre / all-reduce / k_finalize_post); the gossip
    injector's live list is replicated on every rank;
  * full topology: contiguous id slabs, no halo.  Push-sum (gp_fullbin.hip
    k_fbm_send / k_fbm_coarse): every rank bins its messages {sender id, s/2,
    w/2} by destination rank -- its own share included -- into fixed-capacity
    buffers (expected + 12 sigma + 64, an overflow fails), one region per half
    of its slab, exchanged separately, in no particular order (shuffled here); the receiver recomputes every target from the
    sender's Philox draw and folds each receiver's messages by ascending sender
    id.  Gossip (gp_full.hip): deliveries are counts added by the owner.

It never calls the HIP library: it checks the decomposition itself (slab
plan, slot arithmetic, fold order with remote messages, replicated injector)
against the single-process CPU oracle.  Vectorised Philox4x32-10 follows
oracle/srs_py.py (itself pinned by the Random123 known-answer vectors).
"""
from __future__ import annotations

import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
MASK = np.uint64(0xFFFFFFFF)
S_TOPO, S_START, S_GOSSIP, S_PUSHSUM, S_INJECT = 0, 1, 2, 3, 4
DIR_NONE, DIR_RANDOM = 7, 6


def uniform(seed, stream, node, rnd, m):
    """U(m) for arrays of node ids (ctr = (node, round, stream, 0), key = seed)."""
    node = np.asarray(node, dtype=np.uint64)
    c0 = node & MASK
    c1 = np.full_like(node, np.uint64(rnd) & MASK)
    c2 = np.full_like(node, np.uint64(stream))
    c3 = node >> np.uint64(32)
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    for r in range(10):
        if r:
            k0 = (k0 + 0x9E3779B9) & 0xFFFFFFFF
            k1 = (k1 + 0xBB67AE85) & 0xFFFFFFFF
        p0 = M0 * c0
        p1 = M1 * c2
        c0, c1, c2, c3 = ((p1 >> np.uint64(32)) ^ c1 ^ np.uint64(k0)) & MASK, p1 & MASK, \
            ((p0 >> np.uint64(32)) ^ c3 ^ np.uint64(k1)) & MASK, p0 & MASK
    m = np.asarray(m, dtype=np.uint64)
    lo = c0 * m
    hi = c1 * m + (lo >> np.uint64(32))
    return (hi >> np.uint64(32)).astype(np.int64)


def resolve(n, topo):
    if topo in ("line", "full"):
        return n + 1, n, 0
    g = int(round(n ** (1 / 3)))
    while g > 0 and g ** 3 >= n:
        g -= 1
    while g ** 3 < n:
        g += 1
    return g ** 3, g ** 3, g


class Geometry:
    """Implicit neighbours in the reference's slot order (Program.fs:182-191,246-260)."""

    def __init__(self, P, g, topo, seed):
        self.P, self.g, self.topo, self.seed = P, g, topo, seed
        self.ND = 2 if topo == "line" else 6

    def nbr(self, j, d):
        """Neighbour of ids j in direction d, or -1 if absent."""
        j = np.asarray(j, dtype=np.int64)
        if self.topo == "line":
            out = j - 1 if d == 0 else j + 1
            return np.where((out >= 0) & (out < self.P), out, -1)
        g, g2 = self.g, self.g * self.g
        x, y, z = j // g2, (j // g) % g, j % g
        off, ok = [(-g2, x > 0), (g2, x < g - 1), (g, y < g - 1), (-g, y > 0), (1, z < g - 1), (-1, z > 0)][d]
        return np.where(ok, j + off, -1)

    def mask(self, j):
        m = np.zeros(len(j), dtype=np.int64)
        for d in range(self.ND):
            m |= (self.nbr(j, d) >= 0).astype(np.int64) << d
        return m

    def degree(self, j):
        deg = np.zeros(len(j), dtype=np.int64)
        for d in range(self.ND):
            deg += self.nbr(j, d) >= 0
        return deg + (1 if self.topo == "Imp3D" else 0)

    def draw_dir(self, j, stream, rnd):
        """Direction each id in j sends in during round rnd (slot order -> direction)."""
        mask = self.mask(j)
        deg = self.degree(j)
        k = uniform(self.seed, stream, j, rnd, np.maximum(deg, 1))
        out = np.full(len(j), DIR_NONE, dtype=np.int64)
        for d in range(self.ND):              # slot k -> k-th present direction
            has = (mask >> d) & 1 == 1
            take = has & (k == 0) & (out == DIR_NONE)
            out[take] = d
            k = np.where(has & (out == DIR_NONE), k - 1, k)
        if self.topo == "Imp3D":
            out[(out == DIR_NONE) & (deg > 0)] = DIR_RANDOM
        out[deg == 0] = DIR_NONE
        return out


def slab_bounds(P, g, topo, W):
    """gp_api.hip make_bounds."""
    if topo == "line":
        return [P * w // W for w in range(W + 1)], 1
    if topo == "full":
        return [P * w // W for w in range(W + 1)], 0
    return [(g * w // W) * g * g for w in range(W + 1)], g * g


XTILE = 1024  # the lists' tiles: 1024 ids on global multiples (the push-sum tile kernel's TILE)


def region_tiles(lo, nloc, g2, NH, nt):
    """Tile boundaries (relative to lo // XTILE) of the NH exchange regions of a slab
    (gp_round.hip region_tiles): region h holds the planes [x0 + nx h / NH, x0 + nx (h + 1) / NH),
    a tile belonging to the plane it starts in; a slab not made of whole planes is cut
    into equal tile counts."""
    if not g2 or nloc % g2 or lo % g2:
        return [nt * h // NH for h in range(NH + 1)]
    tb, tend = lo // XTILE, (lo + nloc + XTILE - 1) // XTILE
    x0, nx = lo // g2, nloc // g2
    out = []
    for h in range(NH + 1):
        x = x0 + nx * h // NH
        out.append((tb if x <= x0 else min((x * g2 + XTILE - 1) // XTILE, tend)) - tb)
    return out


class ListPlan:
    """Imp3D push-sum over several ranks: the sender-ordered lists (gp_xchg.hpp,
    gp_api.hip build_lists / setup_exchange).  List L_ab = slab a's senders whose
    random edge lands on slab b, in id order, cut into the slab's tiles and NH
    regions of consecutive tiles (region_tiles: whole planes, gp_api.hip XREGIONS = 4);
    every (tile, b) segment starts on a 64-entry
    boundary.  Computed from the global random edges, like every rank of the
    library does for every slab."""

    def __init__(self, P, g, W, bounds, rnd_all, geo, NH=4):
        self.W, self.NH, self.bounds = W, NH, bounds
        owner = np.searchsorted(np.array(bounds[1:-1]), rnd_all, side="right")
        ids = np.arange(P)
        slab = np.searchsorted(np.array(bounds[1:-1]), ids, side="right")
        self.nw = np.zeros((W, NH, W), dtype=np.int64)        # header words of chunk (h, a -> b)
        self.key_local = np.full(P, -1, dtype=np.int64)       # padded index of a sender in its chunk
        self.region = np.zeros(P, dtype=np.int64)
        mu = np.zeros((NH, W, W))
        inv_deg = 1.0 / geo.degree(ids)
        for a in range(W):
            lo, hi = bounds[a], bounds[a + 1]
            t_of = ids[lo:hi] // XTILE - lo // XTILE            # tile of each sender (relative)
            nt = (hi + XTILE - 1) // XTILE - lo // XTILE
            tb = np.array(region_tiles(lo, hi - lo, g * g, NH, nt))
            region_of_tile = np.searchsorted(tb[1:NH], np.arange(nt), side="right")
            h_of = region_of_tile[t_of]
            self.region[lo:hi] = h_of
            np.add.at(mu, (h_of, a, owner[lo:hi]), inv_deg[lo:hi])
            for b in range(W):
                if b == a:
                    continue
                sel = np.nonzero(owner[lo:hi] == b)[0]          # the list, in id order
                cnt = np.bincount(t_of[sel], minlength=nt)
                words = (cnt + 63) // 64
                gw = np.zeros(nt, dtype=np.int64)
                for h in range(NH):
                    in_h = region_of_tile == h
                    gw[in_h] = np.cumsum(words[in_h]) - words[in_h]
                    self.nw[a, h, b] = int(words[in_h].sum())
                first = np.cumsum(cnt) - cnt  # list position of each tile's first entry
                rho = np.arange(len(sel)) - first[t_of[sel]]
                self.key_local[lo + sel] = gw[t_of[sel]] * 64 + rho
        # capacities per (h, a -> b): expected messages + 12 sigma + 64, at most the edges
        n_edges = np.zeros((NH, W, W))
        for a in range(W):
            lo, hi = bounds[a], bounds[a + 1]
            np.add.at(n_edges, (self.region[lo:hi], a, owner[lo:hi]), 1)
        self.cap = np.minimum(np.ceil(mu + 12.0 * np.sqrt(mu) + 64.0), n_edges).astype(np.int64)
        for a in range(W):
            self.cap[:, a, a] = 0
        self.owner, self.slab = owner, slab

    def hw(self, b, h, a):
        """First header word of chunk (h, a) in b's header region (chunks in (h, a) order)."""
        o = 0
        for hh in range(self.NH):
            for aa in range(self.W):
                if aa == b:
                    continue
                if (hh, aa) == (h, a):
                    return o
                o += int(self.nw[aa, hh, b])
        return o

    def vo(self, b, h, a):
        """First slot of chunk (h, a) in b's vals region (same order)."""
        o = 0
        for hh in range(self.NH):
            for aa in range(self.W):
                if aa == b:
                    continue
                if (hh, aa) == (h, a):
                    return o
                o += int(self.cap[hh, aa, b])
        return o

    def key(self, i):
        """List key of sender i at its destination: 64 * header word + bit (build_lists)."""
        a, b, h = self.slab[i], self.owner[i], self.region[i]
        return np.array([self.hw(bb, hh, aa) * 64 for aa, bb, hh in zip(a, b, h)], dtype=np.int64) + self.key_local[i]


def full_capacity(na, nb, P):
    """Per-pair message capacity of the full-topology exchange (gp_api.hip
    setup_exchange): messages a -> b are at most Binomial(na, nb / (P - 1))."""
    m = na * nb / (P - 1)
    return int(min(np.ceil(m + 12.0 * np.sqrt(m) + 64.0), na))


FB_TB = 12       # gp_fullbin.hpp: fine tiles of 4096 receivers
FBM_KEYS = 192   # gp_fullbin.hip: keys of all ranks' coarse bins together, at most


def full_bin_multi_s1(bounds):
    """Coarse-bin size 2^s1 every rank uses on the full topology (gp_fullbin.hip
    full_bin_multi_s1): the smallest >= a fine tile that keeps all ranks' bins together at
    most FBM_KEYS."""
    s1 = FB_TB
    while True:
        keys = sum(-(-(bounds[b + 1] - bounds[b]) // (1 << s1)) for b in range(len(bounds) - 1))
        if keys <= FBM_KEYS or s1 - FB_TB >= 12:
            return s1
        s1 += 1


def full_bin_multi_cap(n, s1, P):
    """Messages a region of n senders sends to one coarse bin (2^s1 receivers) of any rank,
    at most (gp_fullbin.hip full_bin_multi_cap): Binomial(n, 2^s1 / (P - 1)) + 12 sigma + 64."""
    m = n * (1 << s1) / max(P - 1, 1)
    return int(min(np.ceil(m + 12.0 * np.sqrt(m) + 64.0), n))


def full_region(n, NH, h):
    """Region h of NH of a slab of n ids (gp_api.hip full_region): fine tiles [t0, t1),
    local sender ids [s0, s1)."""
    nt = -(-n // (1 << FB_TB))
    t0, t1 = nt * h // NH, nt * (h + 1) // NH
    return min(n, t0 << FB_TB), min(n, t1 << FB_TB)


def full_target(i, k):
    """Slot k of node i on the full topology: the k-th of all j != i (Program.fs:211-216)."""
    return np.where(k < i, k, k + 1)


class RankSim:
    """One rank's slab, advanced in synchronous rounds through the exchange plan."""

    def __init__(self, n, topo, alg, seed, rank, world, dist):
        self.topo, self.alg, self.seed, self.rank, self.W, self.dist = topo, alg, seed, rank, world, dist
        self.P, self.T, self.g = resolve(n, topo)
        self.G = Geometry(self.P, self.g, topo, seed)
        self.bounds, self.H = slab_bounds(self.P, self.g, topo, world)
        self.lo, self.hi = self.bounds[rank], self.bounds[rank + 1]
        self.ext_lo = self.lo - self.H if rank > 0 else self.lo
        self.ext_hi = self.hi + self.H if rank < world - 1 else self.hi
        self.ids = np.arange(self.lo, self.hi, dtype=np.int64)
        self.seed_node = int(uniform(seed, S_START, np.array([0]), 0, self.T)[0])
        n_ext = self.ext_hi - self.ext_lo
        self.dir = np.full(n_ext, DIR_NONE, dtype=np.int64)      # direction of the current round (ext)
        self.round = 0
        self.alerts_total = 0
        self.done = False
        if topo == "Imp3D":
            self._build_inlists()
        if alg == "push-sum":
            self.s = np.arange(self.ext_lo, self.ext_hi, dtype=np.float64)
            self.w = np.ones(n_ext)
            self.active = np.zeros(n_ext, dtype=bool)
            self.cnt = np.ones(self.hi - self.lo, dtype=np.int64)
            self.conv = np.zeros(self.hi - self.lo, dtype=bool)
            if self.lo <= self.seed_node < self.hi:
                self.active[self.seed_node - self.ext_lo] = True
                if topo != "full":
                    self.dir[self.seed_node - self.ext_lo] = self.G.draw_dir(np.array([self.seed_node]), S_PUSHSUM, 0)[0]
            self.active_total = 1
        else:
            self.c = np.zeros(self.hi - self.lo, dtype=np.int64)
            if self.lo <= self.seed_node < self.hi and topo != "full":
                self.dir[self.seed_node - self.ext_lo] = self.G.draw_dir(np.array([self.seed_node]), S_GOSSIP, 0)[0]
            self.live = list(range(self.T)) if topo != "full" else None
        self._exchange(0)
        if alg == "gossip":
            self._prepare_injector(0)

    # ---------------------------------------------------------------- topology
    def _build_inlists(self):
        P = self.P
        rnd_all = uniform(self.seed, S_TOPO, np.arange(P), 0, P - 1)   # Program.fs:259
        order = np.argsort(rnd_all, kind="stable")                     # senders ascending per receiver
        off_all = np.zeros(P + 1, dtype=np.int64)
        np.add.at(off_all, rnd_all + 1, 1)
        off_all = np.cumsum(off_all)
        inv = np.empty(P, dtype=np.int64)
        inv[order] = np.arange(P)
        edge0 = off_all[self.bounds]
        self.in_off = off_all[self.lo:self.hi + 1] - edge0[self.rank]
        self.in_src = order[edge0[self.rank]:edge0[self.rank + 1]]
        self.rnd = rnd_all[self.lo:self.hi]
        self.owner = np.searchsorted(np.array(self.bounds[1:-1]), self.rnd, side="right")
        # slot of each local sender's message in its target owner's in-edge array (k_make_pos)
        self.pos = inv[self.lo:self.hi] - edge0[self.owner]
        ne = len(self.in_src)
        self.rtag = np.full(ne, -1, dtype=np.int64)
        self.rmsg = np.zeros((ne, 2))
        self.plan = None
        if self.alg == "push-sum" and self.W > 1:  # sender-ordered lists (build_lists)
            self.plan = ListPlan(P, self.g, self.W, self.bounds, rnd_all, self.G)
            src = self.in_src
            remote = (src < self.lo) | (src >= self.hi)
            self.rk = np.zeros(ne, dtype=np.int64)
            if remote.any():
                self.rk[remote] = self.plan.key(src[remote])

    def _local(self, ids):
        return ids - self.ext_lo

    # ---------------------------------------------------------------- exchange
    def _exchange(self, rn):
        """Halo refresh + random-edge messages for round rn (state already in place)."""
        import torch
        if self.topo == "full":  # the full topology's exchange is inside the round
            return
        d = self.dist
        fields = [self.dir] + ([self.s, self.w, self.active.astype(np.float64)] if self.alg == "push-sum" else [])
        H = self.H
        if self.W > 1:
            lo_l, hi_l = self.lo - self.ext_lo, self.hi - self.ext_lo
            out = {}
            if self.rank > 0:
                out[self.rank - 1] = [f[lo_l:lo_l + H].astype(np.float64) for f in fields]
            if self.rank < self.W - 1:
                out[self.rank + 1] = [f[hi_l - H:hi_l].astype(np.float64) for f in fields]
            got = [None] * self.W
            d.all_gather_object(got, out)
            for src, payload in enumerate(got):
                if self.rank not in payload:
                    continue
                for f, v in zip(fields, payload[self.rank]):
                    if src == self.rank - 1:
                        f[:H] = v.astype(f.dtype)
                    else:
                        f[hi_l:hi_l + H] = v.astype(f.dtype)
            if self.alg == "push-sum":
                self.active = fields[3].astype(bool)
        if self.topo == "Imp3D" and self.alg == "gossip":
            # counts for round rn: local random-edge sends at their targets (k_gossip_col)
            mydir = self.dir[self._local(self.ids)]
            self.rq = np.zeros(self.hi - self.lo, dtype=np.int64)
            mine = (mydir == DIR_RANDOM) & (self.owner == self.rank)
            np.add.at(self.rq, self.rnd[mine] - self.lo, 1)
        if self.topo == "Imp3D" and self.W > 1 and self.plan is not None:
            self._exchange_lists()
        elif self.topo == "Imp3D" and self.W > 1:
            mydir = self.dir[self._local(self.ids)]
            send = (mydir == DIR_RANDOM) & (self.owner != self.rank)
            packets = {}
            for p in range(self.W):
                sel = send & (self.owner == p)
                if self.alg == "push-sum":
                    li = self._local(self.ids[sel])
                    packets[p] = (self.pos[sel], self.s[li], self.w[li])
                else:  # counts: the target's id local to its owner
                    packets[p] = (self.rnd[sel] - self.bounds[p],)
            got = [None] * self.W
            d.all_gather_object(got, packets)
            for src, pk in enumerate(got):
                if src == self.rank:
                    continue
                msg = pk[self.rank]
                if self.alg == "push-sum":
                    self.rtag[msg[0]] = rn
                    self.rmsg[msg[0], 0] = msg[1]
                    self.rmsg[msg[0], 1] = msg[2]
                else:
                    np.add.at(self.rq, msg[0], 1)
        _ = torch  # gloo transport via torch.distributed

    def _exchange_lists(self):
        """k_list_pack + the transfer: per region h and destination d, one header word
        {mask, base} per 64 list entries and the used entries' (s, w) compacted in list
        order (the library reserves each tile's run with an atomic, so runs land in any
        order; the header's base says where -- here in tile order)."""
        pl, me, W = self.plan, self.rank, self.W
        mydir = self.dir[self._local(self.ids)]
        used_all = (mydir == DIR_RANDOM) & (self.owner != me)
        out = {}
        for d in range(W):
            if d == me:
                continue
            for h in range(pl.NH):
                sel = np.nonzero((self.owner == d) & (pl.region[self.ids] == h))[0]
                kl = pl.key_local[self.ids[sel]]
                used = used_all[sel]
                nw = int(pl.nw[me, h, d])
                mask = np.zeros(nw, dtype=np.uint64)
                np.bitwise_or.at(mask, kl[used] >> 6, np.left_shift(np.uint64(1), (kl[used] & 63).astype(np.uint64)))
                per_word = np.bincount(kl[used] >> 6, minlength=nw)[:nw]
                base = pl.vo(d, h, me) + (np.cumsum(per_word) - per_word).astype(np.int64)
                order = np.argsort(kl[used], kind="stable")            # list order
                li = self._local(self.ids[sel][used][order])
                vals = np.stack([self.s[li], self.w[li]], axis=1) if len(li) else np.zeros((0, 2))
                out[(d, h)] = (mask, base, vals)
        got = [None] * W
        self.dist.all_gather_object(got, out)
        # this rank's receive region: header words and slots of every chunk (h, a), (h, a) order
        hdr_mask, hdr_base, vals = [], [], []
        for h in range(pl.NH):
            for a in range(W):
                if a == me:
                    continue
                m, b, v = got[a][(me, h)]
                hdr_mask.append(m)
                hdr_base.append(b)
                slot = np.zeros((int(pl.cap[h, a, me]), 2))
                slot[:len(v)] = v
                vals.append(slot)
        self.xmask = np.concatenate(hdr_mask) if hdr_mask else np.zeros(0, dtype=np.uint64)
        self.xbase = np.concatenate(hdr_base) if hdr_base else np.zeros(0, dtype=np.int64)
        self.xvals = np.concatenate(vals) if vals else np.zeros((0, 2))

    def _list_lookup(self, k):
        """Receiver side (the round kernel's in-edge pass): did the remote sender with list
        key k use its edge, and where is its message?"""
        w, bit = k >> 6, (k & 63).astype(np.uint64)
        m = self.xmask[w]
        sent = ((m >> bit) & np.uint64(1)) == 1
        below = m & ((np.uint64(1) << bit) - np.uint64(1))
        pc = np.array([bin(int(x)).count("1") for x in below], dtype=np.int64)
        return sent, self.xbase[w] + pc

    def _allreduce(self, vals):
        import torch
        t = torch.tensor(vals, dtype=torch.int64)
        if self.W > 1:
            self.dist.all_reduce(t)
        return [int(v) for v in t.tolist()]

    # ---------------------------------------------------------------- rounds
    def _random_in(self, r):
        """Per local in-edge: did the sender use its random edge in round r?"""
        src = self.in_src
        local = (src >= self.lo) & (src < self.hi)
        sent = np.zeros(len(src), dtype=bool)
        sent[local] = self.dir[self._local(src[local])] == DIR_RANDOM
        if self.plan is not None:  # push-sum: the received lists
            self.rslot = np.zeros(len(src), dtype=np.int64)
            if (~local).any():
                sent[~local], self.rslot[~local] = self._list_lookup(self.rk[~local])
        else:
            sent[~local] = self.rtag[~local] == r
        return sent, local

    def _pushsum_round(self):
        r = self.round
        j = self.ids
        lj = self._local(j)
        deg = self.G.degree(j)
        act = self.active[lj]
        halve = act & (deg > 0)
        acc_s = np.where(halve, self.s[lj] * 0.5, self.s[lj])
        acc_w = np.where(halve, self.w[lj] * 0.5, self.w[lj])
        recv = np.zeros(len(j), dtype=bool)
        for d in range(self.G.ND):            # lattice slots in the receiver's order
            n = self.G.nbr(j, d)
            ok = n >= 0
            ln = self._local(np.where(ok, n, self.lo))
            hit = ok & (self.dir[ln] == (d ^ 1))
            acc_s = np.where(hit, acc_s + self.s[ln] * 0.5, acc_s)
            acc_w = np.where(hit, acc_w + self.w[ln] * 0.5, acc_w)
            recv |= hit
        if self.topo == "Imp3D":              # random edges, ascending sender
            sent, local = self._random_in(r)
            val_s = np.zeros(len(sent))
            val_w = np.zeros(len(sent))
            ls = self._local(self.in_src[local])
            val_s[local], val_w[local] = self.s[ls], self.w[ls]
            if self.plan is not None:
                rs = np.where(sent & ~local, self.rslot, 0)
                val_s[~local], val_w[~local] = self.xvals[rs[~local], 0], self.xvals[rs[~local], 1]
            else:
                val_s[~local], val_w[~local] = self.rmsg[~local, 0], self.rmsg[~local, 1]
            indeg = np.diff(self.in_off)
            for k in range(int(indeg.max()) if len(indeg) else 0):
                has = indeg > k
                e = np.where(has, self.in_off[:-1] + k, 0)
                hit = has & sent[e]
                acc_s = np.where(hit, acc_s + val_s[e] * 0.5, acc_s)
                acc_w = np.where(hit, acc_w + val_w[e] * 0.5, acc_w)
                recv |= hit
        r_old = self.s[lj] / self.w[lj]
        r_new = acc_s / acc_w
        upd = recv & ~self.conv
        self.cnt = np.where(upd, np.where(np.abs(r_new - r_old) > 1e-10, 0, self.cnt + 1), self.cnt)
        newc = upd & (self.cnt == 3)
        self.conv |= newc
        newly = recv & ~act
        self.active[lj] |= recv
        self.s[lj], self.w[lj] = acc_s, acc_w
        nd = self.G.draw_dir(j, S_PUSHSUM, r + 1)
        self.dir[:] = DIR_NONE
        self.dir[lj] = np.where(self.active[lj] & (deg > 0), nd, DIR_NONE)
        self._exchange(r + 1)
        alerts, na, _ = self._allreduce([int(newc.sum()), int(newly.sum()), 0])
        self.active_total += na
        return alerts

    def _prepare_injector(self, rn):
        """Injector pick for round rn on the replicated live list (Program.fs:150-159)."""
        self.inj = -1
        if self.live is None or not self.live:
            self._allreduce([0, 0, 0])
            return
        t = self.live[int(uniform(self.seed, S_INJECT, np.array([0]), rn, len(self.live))[0])]
        mine = self.lo <= t < self.hi and self.c[t - self.lo] >= 11
        conv = self._allreduce([0, 0, int(mine)])[2]
        if conv:
            self.live.remove(t)
        else:
            self.inj = t

    def _gossip_round(self):
        r = self.round
        j = self.ids
        lj = self._local(j)
        conv = self.c >= 11
        inc = np.zeros(len(j), dtype=np.int64)
        for d in range(self.G.ND):
            n = self.G.nbr(j, d)
            ok = n >= 0
            ln = self._local(np.where(ok, n, self.lo))
            inc += ok & (self.dir[ln] == (d ^ 1))
        if self.topo == "Imp3D":  # random-edge rumours, counted a round ahead (local + exchanged)
            inc += self.rq
        if self.lo <= self.inj < self.hi:
            inc[self.inj - self.lo] += 1
        inc[conv] = 0                                   # dropped at converged receivers (Program.fs:87)
        alerts_local = int(((self.c <= 10) & (self.c + inc > 10) & (inc > 0)).sum())
        self.c += inc
        active = ((j == self.seed_node) | (self.c >= 1)) & (self.c <= 10)
        nd = self.G.draw_dir(j, S_GOSSIP, r + 1)
        deg = self.G.degree(j)
        self.dir[:] = DIR_NONE
        self.dir[lj] = np.where(active & (deg > 0), nd, DIR_NONE)
        self._exchange(r + 1)
        alerts = self._allreduce([alerts_local, 0, 0])[0]
        self._prepare_injector(r + 1)
        return alerts

    # ---------------------------------------------------------------- full topology
    def _full_exchange(self, targets, payload):
        """Gossip deliveries (targets) -> this rank's receivers: per-destination
        segments, capacity-checked, concatenated by source rank (counts are
        order-independent)."""
        order = np.argsort(targets, kind="stable")
        t = targets[order]
        pl = [p[order] for p in payload]
        cuts = np.searchsorted(t, np.array(self.bounds), side="left")
        packets = {}
        for b in range(self.W):
            seg = slice(cuts[b], cuts[b + 1])
            if b != self.rank:
                cap = full_capacity(self.hi - self.lo, self.bounds[b + 1] - self.bounds[b], self.P)
                assert cuts[b + 1] - cuts[b] <= cap, "full-topology exchange capacity exceeded"
            packets[b] = (t[seg] - self.bounds[b],) + tuple(x[seg] for x in pl)
        got = [None] * self.W
        if self.W > 1:
            self.dist.all_gather_object(got, packets)
        else:
            got = [packets]
        parts = [got[src][self.rank] for src in range(self.W)]  # ascending source rank
        tt = np.concatenate([p[0] for p in parts])
        cols = [np.concatenate([p[1 + q] for p in parts]) for q in range(len(payload))]
        o2 = np.argsort(tt, kind="stable")
        return tt[o2], [c[o2] for c in cols]

    def _full_pushsum_exchange(self, snd, t, payload):
        """Push-sum messages -> this rank's receivers (gp_fullbin.hip several ranks,
        gp_api.hip launch_round_full_multi, round 6): the senders of each of the slab's two
        exchange regions (whole fine tiles, full_region) are binned by destination rank and
        the destination's coarse bin (2^s1 receivers, the same size on every rank) in
        arbitrary order into fixed-capacity bins (own share included), which are exchanged
        per region; the receiver recomputes the targets and puts each receiver's messages in
        ascending sender order.  Returns local receiver ids and payload columns."""
        owner = np.searchsorted(np.array(self.bounds), t, side="right") - 1
        rng = np.random.default_rng(self.round * 7919 + self.rank)  # buffer order is arbitrary
        n = self.hi - self.lo
        s1 = full_bin_multi_s1(self.bounds)
        parts = []
        for h in range(2):
            r0, r1 = full_region(n, 2, h)
            h_lo, h_hi = self.lo + r0, self.lo + r1
            cap = full_bin_multi_cap(h_hi - h_lo, s1, self.P)
            packets = {}
            for b in range(self.W):
                sel = np.nonzero((owner == b) & (snd >= h_lo) & (snd < h_hi))[0]
                if len(sel):
                    per_bin = np.bincount((t[sel] - self.bounds[b]) >> s1)
                    assert per_bin.max() <= cap, "exchange bin capacity exceeded"
                sel = rng.permutation(sel)
                packets[b] = (snd[sel],) + tuple(p[sel] for p in payload)
            got = [None] * self.W
            if self.W > 1:
                self.dist.all_gather_object(got, packets)
            else:
                got = [packets]
            parts += [got[src][self.rank] for src in range(self.W)]
        src = np.concatenate([p[0] for p in parts]).astype(np.int64)
        cols = [np.concatenate([p[1 + q] for p in parts]) for q in range(len(payload))]
        tt = full_target(src, uniform(self.seed, S_PUSHSUM, src, self.round, self.P - 1)) - self.lo
        o = np.lexsort((src, tt))  # by receiver, then ascending sender: the canonical fold order
        return tt[o], [c[o] for c in cols] + [src[o]]

    def _full_pushsum_round(self):
        r = self.round
        j = self.ids
        lj = self._local(j)
        act = self.active[lj]
        snd = j[act] if self.P > 1 else j[:0]
        t = full_target(snd, uniform(self.seed, S_PUSHSUM, snd, r, self.P - 1))
        li = self._local(snd)
        tt, (ms, mw, src) = self._full_pushsum_exchange(snd, t, [self.s[li] * 0.5, self.w[li] * 0.5])
        halve = act & (self.P > 1)
        acc_s = np.where(halve, self.s[lj] * 0.5, self.s[lj])
        acc_w = np.where(halve, self.w[lj] * 0.5, self.w[lj])
        recv = np.zeros(len(j), dtype=bool)
        if len(tt):
            same = np.concatenate([[False], tt[1:] == tt[:-1]])
            assert np.all(src[1:][same[1:]] > src[:-1][same[1:]]), "senders not ascending per receiver"
            first = np.concatenate([[True], tt[1:] != tt[:-1]])
            rank_in = np.arange(len(tt)) - np.maximum.accumulate(np.where(first, np.arange(len(tt)), 0))
            for k in range(int(rank_in.max()) + 1):     # k-th message of every receiver, in order
                sel = rank_in == k
                rcv = tt[sel]
                acc_s[rcv] = acc_s[rcv] + ms[sel]
                acc_w[rcv] = acc_w[rcv] + mw[sel]
                recv[rcv] = True
        r_old = self.s[lj] / self.w[lj]
        r_new = acc_s / acc_w
        upd = recv & ~self.conv
        self.cnt = np.where(upd, np.where(np.abs(r_new - r_old) > 1e-10, 0, self.cnt + 1), self.cnt)
        newc = upd & (self.cnt == 3)
        self.conv |= newc
        newly = recv & ~act
        self.active[lj] |= recv
        self.s[lj], self.w[lj] = acc_s, acc_w
        alerts, na, _ = self._allreduce([int(newc.sum()), int(newly.sum()), 0])
        self.active_total += na
        return alerts

    def _full_gossip_round(self):
        r = self.round
        j = self.ids
        active = ((j == self.seed_node) | (self.c >= 1)) & (self.c <= 10)
        snd = j[active] if self.P > 1 else j[:0]
        t = full_target(snd, uniform(self.seed, S_GOSSIP, snd, r, self.P - 1))
        tt, _ = self._full_exchange(t, [])
        inc = np.bincount(tt, minlength=len(j)).astype(np.int64)
        inc[self.c >= 11] = 0                           # dropped at converged receivers (Program.fs:87)
        alerts_local = int(((self.c <= 10) & (self.c + inc > 10) & (inc > 0)).sum())
        self.c += inc
        return self._allreduce([alerts_local, 0, 0])[0]

    def step(self, nrounds):
        out = []
        while len(out) < nrounds and not self.done:
            if self.topo == "full":
                a = self._full_gossip_round() if self.alg == "gossip" else self._full_pushsum_round()
            else:
                a = self._gossip_round() if self.alg == "gossip" else self._pushsum_round()
            out.append(a)
            self.alerts_total += a
            self.round += 1
            if self.alerts_total >= self.T:
                self.done = True
        return out

    def state(self):
        """This rank's slab: (lo, c or None, s, w, flags) in the library's flag encoding."""
        lj = self._local(self.ids)
        if self.alg == "gossip":
            act = ((self.ids == self.seed_node) | (self.c >= 1)) & (self.c <= 10)
            flags = act.astype(np.uint8) | ((self.c >= 11).astype(np.uint8) << 1)
            return self.lo, self.c.astype(np.int32), None, None, flags
        flags = self.active[lj].astype(np.uint8) | (self.conv.astype(np.uint8) << 1) | \
            (self.cnt.astype(np.uint8) << 2)
        return self.lo, None, self.s[lj].copy(), self.w[lj].copy(), flags
