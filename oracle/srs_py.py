"""Pure-Python restatement of SRS v1 -- the second, independent oracle.

TEST INFRASTRUCTURE ONLY: imported by tests/ (and the golden-fixture script)
to cross-check the C oracle (oracle/srs_oracle.c) on small populations.  It is
never imported by the product package.

It is written as literally as practical against the reference
(/root/reference/Project2/Program.fs, cited as Program.fs:N): neighbour arrays
are built with the same loops as Program.fs:180-261, messages are explicit
(sender, target) records, and every receiver folds its inbox in the canonical
order of SURVEY.md Appendix B.  Parity with the reference itself is "parity
unpinned" (the reference is asynchronous, seeds System.Random from the clock
and ships no tests); Philox is pinned by the Random123 known-answer vectors.
Loops are pure Python: keep P below ~1e4.
"""
from __future__ import annotations

M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = 0xFFFFFFFF

TOPOLOGIES = {"line": 0, "full": 1, "3D": 2, "Imp3D": 3}
ALGORITHMS = {"gossip": 0, "push-sum": 1}
STREAM_TOPO, STREAM_START, STREAM_GOSSIP, STREAM_PUSHSUM, STREAM_INJECT = range(5)


def philox4x32_10(ctr, key):
    """Random123 Philox4x32, 10 rounds (replaces System.Random, SRS D2)."""
    c0, c1, c2, c3 = (int(v) & MASK for v in ctr)
    k0, k1 = (int(v) & MASK for v in key)
    for rnd in range(10):
        if rnd:
            k0 = (k0 + W0) & MASK
            k1 = (k1 + W1) & MASK
        p0 = M0 * c0
        p1 = M1 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & MASK, p1 & MASK, ((p0 >> 32) ^ c3 ^ k1) & MASK, p0 & MASK
    return c0, c1, c2, c3


def uniform(seed, stream, node, rnd, m):
    """U(m) = floor(((y << 32) | x) * m / 2**64) from ctr = (node, round, stream, node >> 32)."""
    x, y, _, _ = philox4x32_10((node & MASK, rnd, stream, node >> 32), (seed & MASK, seed >> 32))
    return (((y << 32) | x) * m) >> 64


def icbrt_ceil(n):
    """Exact ceil(cbrt(n)); Program.fs:239-240 uses Math.Cbrt + ceil (libm-dependent, Q3)."""
    if n <= 0:
        return 0
    g = int(round(n ** (1.0 / 3.0)))
    while g > 0 and g ** 3 >= n:
        g -= 1
    while g ** 3 < n:
        g += 1
    return g


def resolve(n, topology):
    """(P, T, g): Program.fs:170-171 spawns nodes+1 actors, scheduler stops at `nodes`
    alerts (Program.fs:53); 3D/Imp3D round nodes up to g^3 (Program.fs:239)."""
    if n < 1:
        raise ValueError("num_nodes must be >= 1")
    if topology in ("line", "full"):
        return n + 1, n, 0
    if topology in ("3D", "Imp3D"):
        g = icbrt_ceil(n)
        return g ** 3, g ** 3, g
    raise ValueError(topology)


def build_neighbours(P, g, topology, seed):
    """Neighbour arrays exactly as Program.fs builds them.  Returns (nbrs, n_lattice)
    where n_lattice[i] counts the leading lattice slots (the rest is the Imp3D
    random slot, or every slot for full)."""
    nbrs, nlat = [], []
    if topology == "line":  # Program.fs:182-191
        nodes = P - 1
        for i in range(0, nodes + 1):
            if i == 0:
                arr = [i + 1]
            elif i == nodes:
                arr = [i - 1]
            else:
                arr = [i - 1, i + 1]
            nbrs.append(arr)
            nlat.append(len(arr))
    elif topology == "full":  # Program.fs:211-216
        for i in range(P):
            nbrs.append([j for j in range(P) if j != i])
            nlat.append(0)
    else:  # Program.fs:242-261
        nbrs = [None] * P
        nlat = [0] * P
        grid = g
        for i in range(grid):
            for j in range(grid):
                for k in range(grid):
                    arr = []
                    if i - 1 >= 0:
                        arr.append((i - 1) * (grid * grid) + j * grid + k)
                    if i + 1 < grid:
                        arr.append((i + 1) * (grid * grid) + j * grid + k)
                    if j + 1 < grid:
                        arr.append(i * (grid * grid) + (j + 1) * grid + k)
                    if j - 1 >= 0:
                        arr.append(i * (grid * grid) + (j - 1) * grid + k)
                    if k + 1 < grid:
                        arr.append(i * (grid * grid) + j * grid + k + 1)
                    if k - 1 >= 0:
                        arr.append(i * (grid * grid) + j * grid + k - 1)
                    idx = i * (grid * grid) + j * grid + k
                    nlat[idx] = len(arr)
                    if topology != "3D":  # Program.fs:258-260, Random().Next(0, nodes-1)
                        arr.append(uniform(seed, STREAM_TOPO, idx, 0, P - 1))
                    nbrs[idx] = arr
    return nbrs, nlat


class PySim:
    """Literal synchronous-round simulator (SRS v1)."""

    def __init__(self, num_nodes, topology, algorithm, seed=1):
        self.topology, self.algorithm, self.seed = topology, algorithm, seed
        self.P, self.T, self.g = resolve(num_nodes, topology)
        self.nbrs, self.nlat = build_neighbours(self.P, self.g, topology, seed)
        # choice = Random().Next(0, nodes) (Program.fs:193,221,263)
        self.seed_node = uniform(seed, STREAM_START, 0, 0, self.T)
        self.round = 0
        self.alerts_total = 0
        self.done = False
        if algorithm == "gossip":
            self.c = [0] * self.P  # rumours (Program.fs:68)
            # injector list 0..nodes-1 (Program.fs:147-148), line/3D/Imp3D only
            self.live = list(range(self.T)) if topology != "full" else None
        else:
            self.s = [float(i) for i in range(self.P)]  # InitialSum (Program.fs:78,174)
            self.w = [1.0] * self.P  # Program.fs:71
            self.cnt = [1] * self.P  # Program.fs:67
            self.conv = [False] * self.P
            self.active = [False] * self.P
            self.active[self.seed_node] = True

    # -- gossip ------------------------------------------------------------
    def _gossip_round(self):
        r = self.round
        conv = [ci >= 11 for ci in self.c]  # dictionary snapshot
        inc = [0] * self.P
        for i in range(self.P):  # Process1, Program.fs:84-89
            ci = self.c[i]
            if not ((i == self.seed_node or ci >= 1) and ci <= 10):
                continue
            deg = len(self.nbrs[i])
            if deg == 0:
                continue
            t = self.nbrs[i][uniform(self.seed, STREAM_GOSSIP, i, r, deg)]
            if not conv[t]:
                inc[t] += 1
        if self.live is not None and len(self.live) > 0:  # Actor2, Program.fs:150-159
            k = uniform(self.seed, STREAM_INJECT, 0, r, len(self.live))
            t = self.live[k]
            if conv[t]:
                self.live.remove(t)
            else:
                inc[t] += 1
        alerts = 0
        for j in range(self.P):  # Process2, Program.fs:91-98
            if inc[j]:
                if self.c[j] <= 10 < self.c[j] + inc[j]:
                    alerts += 1
                self.c[j] += inc[j]
        return alerts

    # -- push-sum ----------------------------------------------------------
    def _pushsum_round(self):
        r = self.round
        inbox = [[] for _ in range(self.P)]
        msg = {}
        for i in range(self.P):  # send half (Program.fs:102-106,125-128)
            if not self.active[i]:
                continue
            deg = len(self.nbrs[i])
            if deg == 0:
                continue
            k = uniform(self.seed, STREAM_PUSHSUM, i, r, deg)
            t = self.nbrs[i][k]
            msg[i] = (self.s[i] * 0.5, self.w[i] * 0.5)
            inbox[t].append((i, k < self.nlat[i]))
        alerts = 0
        news, neww = list(self.s), list(self.w)
        for j in range(self.P):
            s0, w0 = self.s[j], self.w[j]
            halve = self.active[j] and len(self.nbrs[j]) > 0
            acc_s = s0 * 0.5 if halve else s0
            acc_w = w0 * 0.5 if halve else w0
            if inbox[j]:
                lattice = [snd for snd, lat in inbox[j] if lat]
                rand = sorted(snd for snd, lat in inbox[j] if not lat)
                ordered = [n for n in self.nbrs[j][: self.nlat[j]] if n in lattice] + rand
                assert len(ordered) == len(inbox[j])
                for snd in ordered:
                    acc_s = acc_s + msg[snd][0]
                    acc_w = acc_w + msg[snd][1]
                r_old = s0 / w0
                r_new = acc_s / acc_w
                if not self.conv[j]:  # Program.fs:114-123
                    self.cnt[j] = 0 if abs(r_new - r_old) > 1e-10 else self.cnt[j] + 1
                    if self.cnt[j] == 3:
                        self.conv[j] = True
                        alerts += 1
                self.active[j] = True
            news[j], neww[j] = acc_s, acc_w
        self.s, self.w = news, neww
        return alerts

    def step(self, nrounds):
        """Run up to nrounds rounds (stops once cumulative alerts reach T, Program.fs:53)."""
        out = []
        while len(out) < nrounds and not self.done:
            a = self._gossip_round() if self.algorithm == "gossip" else self._pushsum_round()
            out.append(a)
            self.alerts_total += a
            self.round += 1
            if self.alerts_total >= self.T:
                self.done = True
        return out

    def flags(self):
        if self.algorithm == "gossip":
            return [int((i == self.seed_node or ci >= 1) and ci <= 10) | (int(ci >= 11) << 1)
                    for i, ci in enumerate(self.c)]
        return [int(a) | (int(cv) << 1) | (cn << 2) for a, cv, cn in zip(self.active, self.conv, self.cnt)]


__all__ = ["PySim", "philox4x32_10", "uniform", "icbrt_ceil", "resolve", "build_neighbours",
           "TOPOLOGIES", "ALGORITHMS"]
