/*
 * srs_oracle.c -- CPU oracle: SRS v1 restatement of the reference hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see srs_oracle.h for who may load it, and for the
 * parity status: end-to-end parity with the asynchronous reference is
 * "parity unpinned"; Philox KATs and Program.fs neighbour orders are pinned).
 *
 * Build: gcc -O2 -fopenmp -ffp-contract=off -fPIC -shared (see Makefile).
 * -ffp-contract=off is mandatory: the HIP kernels are built the same way and
 * the push-sum fold must round identically.
 *
 * Every function cites the Program.fs lines it restates
 * (Program.fs = /root/reference/Project2/Program.fs).
 */
#include "srs_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define NONE_U32 0xFFFFFFFFu
#define RANDOM_KEY_BASE (1ull << 40)

/* ---------------------------------------------------------------- Philox */
/* Random123 Philox4x32 with 10 rounds.  Replaces System.Random
 * (Program.fs:86,103,128,130,152,193,221,259,263), SRS deviation D2. */
void or_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

uint32_t or_uniform(uint64_t seed, uint32_t stream, uint64_t node, uint32_t round, uint32_t m) {
    uint32_t ctr[4] = {(uint32_t)node, round, stream, (uint32_t)(node >> 32)};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t o[4];
    or_philox4x32_10(ctr, key, o);
    /* floor(((y<<32)|x) * m / 2^64) via 128-bit product */
    unsigned __int128 v = ((unsigned __int128)(((uint64_t)o[1] << 32) | o[0])) * m;
    return (uint32_t)(v >> 64);
}

/* Program.fs:239-240 rounds nodes up to a cube with Math.Cbrt + ceil; that is
 * platform-libm dependent (glibc cbrt(27) = 3.0000000000000004 -> 4), so SRS v1
 * pins it with an exact integer cube root. */
int64_t or_icbrt_ceil(int64_t n) {
    if (n <= 0) return 0;
    int64_t g = (int64_t)cbrt((double)n);
    while (g > 0 && g * g * g >= n) --g;
    while (g * g * g < n) ++g;
    return g;
}

/* Population rules: Program.fs:170-171 spawns nodes+1 actors and the
 * scheduler stops at `nodes` alerts (Program.fs:53) -> P = n+1, T = n for line
 * and full.  3D/Imp3D: P = T = g^3 (Program.fs:239, SRS D1 drops the
 * unreachable extra actor). */
int or_resolve(int64_t n, int topology, int64_t* P, int64_t* T, int64_t* g) {
    if (n < 1) return -1;
    if (topology == OR_LINE || topology == OR_FULL) {
        *P = n + 1; *T = n; *g = 0;
    } else if (topology == OR_3D || topology == OR_IMP3D) {
        int64_t gg = or_icbrt_ceil(n);
        *g = gg; *P = gg * gg * gg; *T = *P;
    } else {
        return -1;
    }
    if (*P > 0xFFFFF000ll) return -1; /* node ids are u32; same limit as GP_MAX_POPULATION */
    return 0;
}

/* ---------------------------------------------------------------- state */
struct or_sim {
    int topo, alg, threads;
    uint64_t seed;
    int64_t n, P, T, g, max_rounds;
    int64_t seed_node;
    int64_t round;          /* next round index */
    int64_t alerts_total;
    int done;
    /* gossip */
    int32_t* c;
    int32_t* inc;
    /* injector (Program.fs:141-163): Fenwick tree over the live id list */
    int32_t* fen;
    uint8_t* removed;
    int64_t live;
    /* push-sum */
    double *s, *w, *s_msg, *w_msg;
    uint8_t *active, *conv, *cnt;
    /* Imp3D random edge (Program.fs:258-260) */
    uint32_t* rnd;
    /* message buckets */
    uint32_t* tgt;
    uint64_t* mkey;
    uint32_t* bcount;   /* P+1 */
    uint32_t* bcursor;  /* P   */
    uint32_t* items;    /* P   */
    /* full push-sum: (target << 32 | sender) keys and the radix sort's second buffer */
    uint64_t* mkey2;
    int64_t* rhist;     /* threads * 65536 digit counters */
};

static int nthreads(const or_sim* s) { return s->threads > 0 ? s->threads : 1; }

/* Lattice neighbours of node i in the reference's slot order
 * (Program.fs:246-257: x-1, x+1, y+1, y-1, z+1, z-1, each only if in range),
 * id = x*g^2 + y*g + z with x = plane i, y = row j, z = column k (Program.fs:242-244,261). */
static int lattice_nbrs(int64_t g, int64_t id, int64_t* out) {
    int64_t g2 = g * g;
    int64_t x = id / g2, y = (id / g) % g, z = id % g;
    int d = 0;
    if (x - 1 >= 0) out[d++] = (x - 1) * g2 + y * g + z;
    if (x + 1 < g) out[d++] = (x + 1) * g2 + y * g + z;
    if (y + 1 < g) out[d++] = x * g2 + (y + 1) * g + z;
    if (y - 1 >= 0) out[d++] = x * g2 + (y - 1) * g + z;
    if (z + 1 < g) out[d++] = x * g2 + y * g + z + 1;
    if (z - 1 >= 0) out[d++] = x * g2 + y * g + z - 1;
    return d;
}

/* Line neighbours (Program.fs:182-191): node 0 -> [1], node nodes -> [nodes-1],
 * else [i-1, i+1]. */
static int line_nbrs(int64_t P, int64_t i, int64_t* out) {
    if (i == 0) { out[0] = 1; return 1; }
    if (i == P - 1) { out[0] = P - 2; return 1; }
    out[0] = i - 1; out[1] = i + 1;
    return 2;
}

static int64_t degree(const or_sim* s, int64_t i) {
    int64_t tmp[7];
    switch (s->topo) {
    case OR_LINE: return line_nbrs(s->P, i, tmp);
    case OR_FULL: return s->P - 1; /* Program.fs:211-216: every j != i */
    case OR_3D: return lattice_nbrs(s->g, i, tmp);
    default: return lattice_nbrs(s->g, i, tmp) + 1;
    }
}

/* Slot k of node i -> target.  *is_random set for the Imp3D random slot and
 * for every full-topology slot (these are folded by ascending sender id);
 * otherwise *lat_key = position of i in the target's own slot list. */
static int64_t slot_target(const or_sim* s, int64_t i, int64_t k, int* is_random) {
    int64_t nb[7];
    int d;
    *is_random = 0;
    switch (s->topo) {
    case OR_LINE:
        line_nbrs(s->P, i, nb);
        return nb[k];
    case OR_FULL:
        *is_random = 1;
        return k < i ? k : k + 1; /* ascending j != i (Program.fs:213-215) */
    case OR_3D:
        lattice_nbrs(s->g, i, nb);
        return nb[k];
    default:
        d = lattice_nbrs(s->g, i, nb);
        if (k == d) { *is_random = 1; return s->rnd[i]; }
        return nb[k];
    }
}

static uint64_t lattice_key(const or_sim* s, int64_t target, int64_t sender) {
    int64_t nb[7];
    int d = (s->topo == OR_LINE) ? line_nbrs(s->P, target, nb) : lattice_nbrs(s->g, target, nb);
    for (int q = 0; q < d; ++q)
        if (nb[q] == sender) return (uint64_t)q;
    return ~0ull; /* unreachable: lattice adjacency is symmetric */
}

int or_neighbors(const or_sim* s, int64_t i, int64_t* out) {
    if (i < 0 || i >= s->P) return -1;
    int64_t deg = degree(s, i);
    if (out) {
        for (int64_t k = 0; k < deg; ++k) {
            int r;
            out[k] = slot_target(s, i, k, &r);
        }
    }
    return (int)deg;
}

/* ---------------------------------------------------------------- Fenwick */
static void fen_add(or_sim* s, int64_t idx, int32_t v) {
    for (int64_t i = idx + 1; i <= s->T; i += i & -i) s->fen[i] += v;
}
/* 0-indexed k-th live id (k < live): smallest idx with prefix(idx+1) > k */
static int64_t fen_kth(const or_sim* s, int64_t k) {
    int64_t pos = 0, step = 1;
    while (step * 2 <= s->T) step *= 2;
    int64_t rem = k;
    for (; step; step >>= 1) {
        if (pos + step <= s->T && s->fen[pos + step] <= rem) {
            pos += step;
            rem -= s->fen[pos];
        }
    }
    return pos; /* 1-based pos+1 is the answer -> 0-based pos */
}

/* ---------------------------------------------------------------- create */
or_sim* or_create(int64_t num_nodes, int topology, int algorithm, uint64_t seed,
                  int64_t max_rounds, int threads) {
    int64_t P, T, g;
    if (or_resolve(num_nodes, topology, &P, &T, &g)) return NULL;
    if (algorithm != OR_GOSSIP && algorithm != OR_PUSHSUM) return NULL;
    or_sim* s = (or_sim*)calloc(1, sizeof(or_sim));
    if (!s) return NULL;
    s->topo = topology; s->alg = algorithm; s->seed = seed;
    s->n = num_nodes; s->P = P; s->T = T; s->g = g;
    s->max_rounds = max_rounds;
#ifdef _OPENMP
    /* default: all cores, except for small populations, whose rounds are too short
     * for a fork-join per loop to pay (and oversubscribe when tests run in parallel) */
    s->threads = threads > 0 ? threads : (P < 262144 ? 1 : omp_get_max_threads());
#else
    (void)threads;
    s->threads = 1;
#endif
    int nt = nthreads(s);
    int ok = 1;
    s->tgt = (uint32_t*)malloc(sizeof(uint32_t) * P);
    ok &= s->tgt != NULL;
    if (topology == OR_IMP3D) {
        s->rnd = (uint32_t*)malloc(sizeof(uint32_t) * P);
        ok &= s->rnd != NULL;
    }
    if (algorithm == OR_GOSSIP) {
        s->c = (int32_t*)calloc(P, sizeof(int32_t));
        s->inc = (int32_t*)calloc(P, sizeof(int32_t));
        ok &= s->c && s->inc;
        if (topology != OR_FULL) {
            s->fen = (int32_t*)calloc(T + 1, sizeof(int32_t));
            s->removed = (uint8_t*)calloc(T, 1);
            ok &= s->fen && s->removed;
        }
    } else {
        s->s = (double*)malloc(sizeof(double) * P);
        s->w = (double*)malloc(sizeof(double) * P);
        s->s_msg = (double*)malloc(sizeof(double) * P);
        s->w_msg = (double*)malloc(sizeof(double) * P);
        s->active = (uint8_t*)calloc(P, 1);
        s->conv = (uint8_t*)calloc(P, 1);
        s->cnt = (uint8_t*)malloc(P);
        s->mkey = (uint64_t*)malloc(sizeof(uint64_t) * P);
        s->bcount = (uint32_t*)malloc(sizeof(uint32_t) * (P + 1));
        s->bcursor = (uint32_t*)malloc(sizeof(uint32_t) * P);
        s->items = (uint32_t*)malloc(sizeof(uint32_t) * P);
        ok &= s->s && s->w && s->s_msg && s->w_msg && s->active && s->conv && s->cnt &&
              s->mkey && s->bcount && s->bcursor && s->items;
        if (topology == OR_FULL) {
            s->mkey2 = (uint64_t*)malloc(sizeof(uint64_t) * P);
            s->rhist = (int64_t*)malloc(sizeof(int64_t) * 65536 * (size_t)nt);
            ok &= s->mkey2 && s->rhist;
        }
    }
    if (!ok) { or_destroy(s); return NULL; }

    /* Imp3D random neighbour: Random().Next(0, nodes-1) -> [0, P-2]
     * (Program.fs:259), one per node, drawn once at build time. */
    if (topology == OR_IMP3D) {
        #pragma omp parallel for num_threads(nt) schedule(static)
        for (int64_t i = 0; i < P; ++i)
            s->rnd[i] = or_uniform(seed, OR_STREAM_TOPO, (uint64_t)i, 0, (uint32_t)(P - 1));
    }
    /* seed choice = Random().Next(0, nodes) (Program.fs:193,221,263) */
    s->seed_node = or_uniform(seed, OR_STREAM_START, 0, 0, (uint32_t)T);

    if (algorithm == OR_GOSSIP) {
        /* rumours = 0 (Program.fs:68); injector list = ids 0..nodes-1
         * (Program.fs:147-148) */
        if (s->fen) {
            for (int64_t i = 1; i <= T; ++i) {
                s->fen[i] += 1;
                int64_t p = i + (i & -i);
                if (p <= T) s->fen[p] += s->fen[i];
            }
            s->live = T;
        }
    } else {
        /* sum = id (InitialSum x, Program.fs:78,174), weight = 1.0
         * (Program.fs:71), count = 1 (Program.fs:67); only the seed is active */
        #pragma omp parallel for num_threads(nt) schedule(static)
        for (int64_t i = 0; i < P; ++i) {
            s->s[i] = (double)i;
            s->w[i] = 1.0;
            s->cnt[i] = 1;
        }
        s->active[s->seed_node] = 1;
    }
    return s;
}

void or_destroy(or_sim* s) {
    if (!s) return;
    free(s->c); free(s->inc); free(s->fen); free(s->removed);
    free(s->s); free(s->w); free(s->s_msg); free(s->w_msg);
    free(s->active); free(s->conv); free(s->cnt);
    free(s->rnd); free(s->tgt); free(s->mkey);
    free(s->bcount); free(s->bcursor); free(s->items);
    free(s->mkey2); free(s->rhist);
    free(s);
}

/* ---------------------------------------------------------------- gossip */
/* One synchronous gossip round (SRS v1 B.3):
 *   Process1 (Program.fs:84-89): a node with 1 <= rumours <= 10 (or the seed
 *   at 0) picks a uniform neighbour and sends iff the target is not converged
 *   in the round-start snapshot (the `dictionary` check, Program.fs:87).
 *   Injector Process1 (Program.fs:150-159): pick uniformly from the live list;
 *   deliver if unconverged, else remove.
 *   Process2 (Program.fs:91-98): the receipt that finds rumours == 10 alerts;
 *   rumours counts every receipt. */
static int64_t gossip_round(or_sim* s) {
    const int64_t P = s->P;
    const uint32_t r = (uint32_t)s->round;
    int nt = nthreads(s);
    #pragma omp parallel for num_threads(nt) schedule(static)
    for (int64_t i = 0; i < P; ++i) {
        int32_t ci = s->c[i];
        int active = (i == s->seed_node || ci >= 1) && ci <= 10;
        if (!active) continue;
        int64_t deg = degree(s, i);
        if (deg <= 0) continue;
        uint32_t k = or_uniform(s->seed, OR_STREAM_GOSSIP, (uint64_t)i, r, (uint32_t)deg);
        int rnd;
        int64_t t = slot_target(s, i, k, &rnd);
        if (s->c[t] < 11) {
            #pragma omp atomic
            s->inc[t] += 1;
        }
    }
    if (s->fen && s->live > 0) {
        uint32_t k = or_uniform(s->seed, OR_STREAM_INJECT, 0, r, (uint32_t)s->live);
        int64_t t = fen_kth(s, k);
        if (s->c[t] >= 11) {
            s->removed[t] = 1;
            fen_add(s, t, -1);
            s->live -= 1;
        } else {
            s->inc[t] += 1;
        }
    }
    int64_t alerts = 0;
    #pragma omp parallel for num_threads(nt) schedule(static) reduction(+ : alerts)
    for (int64_t j = 0; j < P; ++j) {
        int32_t d = s->inc[j];
        if (!d) continue;
        int32_t c0 = s->c[j], c1 = c0 + d;
        if (c0 <= 10 && c1 > 10) alerts += 1;
        s->c[j] = c1;
        s->inc[j] = 0;
    }
    return alerts;
}

/* ---------------------------------------------------------------- push-sum */
static int cmp_key_items(const or_sim* s, uint32_t a, uint32_t b) {
    return s->mkey[a] < s->mkey[b];
}

/* One synchronous push-sum round (SRS v1 B.4), restating MainPushSum
 * (Program.fs:101-131):
 *   send   -- every active node halves (sum, weight) and sends the halves to one
 *             uniform neighbour (Program.fs:104-106,125-128);
 *   receive-- sum += s, weight += w for each message in canonical order
 *             (own half, lattice slots in the receiver's order, then random
 *             / full messages by ascending sender id);
 *   test   -- |s'/w' - s/w| > 1e-10 resets count else count+1; count == 3
 *             converges and alerts (Program.fs:114-123).  SRS D5 compares
 *             against the round-start ratio (the reference's `difference` is
 *             always 0, Q11); D6 keeps converged nodes sending; D7 one test per
 *             round. */
/* v[0..n) <- inclusive prefix sums, in nt contiguous slices (per-slice totals,
 * their exclusive scan, then each slice's running sum) -- the serial scan over
 * P = 1e9 counters was most of a round on a many-core host. */
static void par_inclusive_scan_u32(uint32_t* v, int64_t n, int nt) {
    uint64_t part[1025];
    if (nt > 1024) nt = 1024;
    #pragma omp parallel num_threads(nt)
    {
#ifdef _OPENMP
        const int t = omp_get_thread_num(), T = omp_get_num_threads();
#else
        const int t = 0, T = 1;
#endif
        const int64_t a = n * t / T, b = n * (t + 1) / T;
        uint64_t sum = 0;
        for (int64_t i = a; i < b; ++i) sum += v[i];
        part[t + 1] = sum;
        #pragma omp barrier
        #pragma omp single
        {
            part[0] = 0;
            for (int q = 1; q <= T; ++q) part[q] += part[q - 1];
        }
        uint64_t run = part[t];
        for (int64_t i = a; i < b; ++i) {
            run += v[i];
            v[i] = (uint32_t)run;
        }
    }
}

static int64_t pushsum_round(or_sim* s) {
    const int64_t P = s->P;
    const uint32_t r = (uint32_t)s->round;
    int nt = nthreads(s);

    /* phase 1: senders */
    #pragma omp parallel for num_threads(nt) schedule(static)
    for (int64_t i = 0; i < P; ++i) {
        s->tgt[i] = NONE_U32;
        if (!s->active[i]) continue;
        int64_t deg = degree(s, i);
        if (deg <= 0) continue;
        uint32_t k = or_uniform(s->seed, OR_STREAM_PUSHSUM, (uint64_t)i, r, (uint32_t)deg);
        int rnd;
        int64_t t = slot_target(s, i, k, &rnd);
        s->tgt[i] = (uint32_t)t;
        s->mkey[i] = rnd ? RANDOM_KEY_BASE + (uint64_t)i : lattice_key(s, t, i);
        s->s_msg[i] = s->s[i] * 0.5;
        s->w_msg[i] = s->w[i] * 0.5;
    }
    /* phase 2: bucket messages by receiver (counting sort; order inside a
     * bucket is fixed afterwards by sorting on the unique keys) */
    #pragma omp parallel for num_threads(nt) schedule(static)
    for (int64_t j = 0; j <= P; ++j) s->bcount[j] = 0;
    #pragma omp parallel for num_threads(nt) schedule(static)
    for (int64_t i = 0; i < P; ++i) {
        uint32_t t = s->tgt[i];
        if (t != NONE_U32) {
            #pragma omp atomic
            s->bcount[t + 1] += 1;
        }
    }
    par_inclusive_scan_u32(s->bcount + 1, P, nt);
    #pragma omp parallel for num_threads(nt) schedule(static)
    for (int64_t j = 0; j < P; ++j) s->bcursor[j] = s->bcount[j];
    #pragma omp parallel for num_threads(nt) schedule(static)
    for (int64_t i = 0; i < P; ++i) {
        uint32_t t = s->tgt[i];
        if (t == NONE_U32) continue;
        uint32_t pos;
        #pragma omp atomic capture
        pos = s->bcursor[t]++;
        s->items[pos] = (uint32_t)i;
    }
    /* phase 3: receivers fold in canonical order */
    int64_t alerts = 0;
    #pragma omp parallel for num_threads(nt) schedule(static) reduction(+ : alerts)
    for (int64_t j = 0; j < P; ++j) {
        int halve = s->active[j] && degree(s, j) > 0;
        double s0 = s->s[j], w0 = s->w[j];
        double os = halve ? s0 * 0.5 : s0;
        double ow = halve ? w0 * 0.5 : w0;
        uint32_t b = s->bcount[j], e = s->bcount[j + 1];
        if (b == e) {
            s->s[j] = os; s->w[j] = ow;
            continue;
        }
        for (uint32_t p = b + 1; p < e; ++p) { /* insertion sort by key */
            uint32_t v = s->items[p];
            uint32_t q = p;
            while (q > b && cmp_key_items(s, v, s->items[q - 1])) {
                s->items[q] = s->items[q - 1];
                --q;
            }
            s->items[q] = v;
        }
        double acc_s = os, acc_w = ow;
        for (uint32_t p = b; p < e; ++p) {
            uint32_t i = s->items[p];
            acc_s = acc_s + s->s_msg[i];
            acc_w = acc_w + s->w_msg[i];
        }
        double r_old = s0 / w0;
        double r_new = acc_s / acc_w;
        if (!s->conv[j]) {
            uint8_t cnt = s->cnt[j];
            cnt = (fabs(r_new - r_old) > 1e-10) ? 0 : (uint8_t)(cnt + 1);
            if (cnt == 3) { s->conv[j] = 1; alerts += 1; }
            s->cnt[j] = cnt;
        }
        s->active[j] = 1;
        s->s[j] = acc_s;
        s->w[j] = acc_w;
    }
    return alerts;
}

/* One stable LSD pass on the 16-bit digit at `shift` (parallel: every thread
 * counts and then scatters its own contiguous slice, the per-(digit, thread)
 * offsets keep slices in order, so equal digits keep their input order). */
static void radix_pass(const uint64_t* in, uint64_t* out, int64_t n, int shift, int nt, int64_t* hist) {
    #pragma omp parallel num_threads(nt)
    {
#ifdef _OPENMP
        const int t = omp_get_thread_num();
#else
        const int t = 0;
#endif
        const int64_t a = n * t / nt, b = n * (t + 1) / nt;
        int64_t* h = hist + (size_t)t * 65536;
        memset(h, 0, sizeof(int64_t) * 65536);
        for (int64_t i = a; i < b; ++i) h[(in[i] >> shift) & 0xFFFF] += 1;
        #pragma omp barrier
        #pragma omp single
        {
            int64_t run = 0;
            for (int d = 0; d < 65536; ++d)
                for (int q = 0; q < nt; ++q) {
                    int64_t c = hist[(size_t)q * 65536 + d];
                    hist[(size_t)q * 65536 + d] = run;
                    run += c;
                }
        }
        for (int64_t i = a; i < b; ++i) out[h[(in[i] >> shift) & 0xFFFF]++] = in[i];
    }
}

/* Push-sum round on the full topology (SRS v1 B.4 with Program.fs:209-216's
 * "every j != i"): same rules as pushsum_round, but the messages are grouped by
 * receiver with a stable two-pass radix sort of (target << 32 | sender) keys --
 * the keys are produced in ascending sender order, so every receiver's
 * messages come out by ascending sender id (the canonical fold order) without
 * per-bucket sorting.  Inactive senders carry target 0xFFFFFFFF and sort last. */
static int64_t pushsum_round_full(or_sim* s) {
    const int64_t P = s->P;
    const uint32_t r = (uint32_t)s->round;
    int nt = nthreads(s);
    #pragma omp parallel for num_threads(nt) schedule(static)
    for (int64_t i = 0; i < P; ++i) {
        uint64_t t = NONE_U32;
        if (s->active[i] && P > 1) {
            uint32_t k = or_uniform(s->seed, OR_STREAM_PUSHSUM, (uint64_t)i, r, (uint32_t)(P - 1));
            t = (int64_t)k < i ? k : (uint64_t)k + 1; /* Program.fs:213-215 */
            s->s_msg[i] = s->s[i] * 0.5;
            s->w_msg[i] = s->w[i] * 0.5;
        }
        s->mkey[i] = (t << 32) | (uint64_t)i;
    }
    radix_pass(s->mkey, s->mkey2, P, 32, nt, s->rhist);
    radix_pass(s->mkey2, s->mkey, P, 48, nt, s->rhist);
    uint32_t* head = s->bcount;
    memset(head, 0xFF, sizeof(uint32_t) * P);
    #pragma omp parallel for num_threads(nt) schedule(static)
    for (int64_t p = 0; p < P; ++p) {
        uint32_t t = (uint32_t)(s->mkey[p] >> 32);
        if (t != NONE_U32 && (p == 0 || (uint32_t)(s->mkey[p - 1] >> 32) != t)) head[t] = (uint32_t)p;
    }
    int64_t alerts = 0;
    #pragma omp parallel for num_threads(nt) schedule(static) reduction(+ : alerts)
    for (int64_t j = 0; j < P; ++j) {
        int halve = s->active[j] && P > 1;
        double s0 = s->s[j], w0 = s->w[j];
        double os = halve ? s0 * 0.5 : s0;
        double ow = halve ? w0 * 0.5 : w0;
        uint32_t b = head[j];
        if (b == NONE_U32) {
            s->s[j] = os; s->w[j] = ow;
            continue;
        }
        double acc_s = os, acc_w = ow;
        for (int64_t p = b; p < P && (uint32_t)(s->mkey[p] >> 32) == (uint32_t)j; ++p) {
            uint32_t i = (uint32_t)s->mkey[p];
            acc_s = acc_s + s->s_msg[i];
            acc_w = acc_w + s->w_msg[i];
        }
        double r_old = s0 / w0;
        double r_new = acc_s / acc_w;
        if (!s->conv[j]) {
            uint8_t cnt = s->cnt[j];
            cnt = (fabs(r_new - r_old) > 1e-10) ? 0 : (uint8_t)(cnt + 1);
            if (cnt == 3) { s->conv[j] = 1; alerts += 1; }
            s->cnt[j] = cnt;
        }
        s->active[j] = 1;
        s->s[j] = acc_s;
        s->w[j] = acc_w;
    }
    return alerts;
}

/* ---------------------------------------------------------------- driver */
/* scheduler (Program.fs:41-61): count Alerts, stop when counter = nodes. */
int64_t or_step(or_sim* s, int64_t nrounds, int64_t* alerts_out) {
    int64_t done = 0;
    while (done < nrounds && !s->done) {
        if (s->max_rounds > 0 && s->round >= s->max_rounds) break;
        int64_t a = s->alg == OR_GOSSIP ? gossip_round(s)
                    : s->topo == OR_FULL ? pushsum_round_full(s) : pushsum_round(s);
        if (alerts_out) alerts_out[done] = a;
        s->alerts_total += a;
        s->round += 1;
        done += 1;
        if (s->alerts_total >= s->T) s->done = 1;
    }
    return done;
}

int64_t or_rounds_done(const or_sim* s) { return s->round; }
int64_t or_alerts_total(const or_sim* s) { return s->alerts_total; }
int64_t or_population(const or_sim* s) { return s->P; }
int64_t or_threshold(const or_sim* s) { return s->T; }
int64_t or_seed_node(const or_sim* s) { return s->seed_node; }

/* CPU-baseline timing only (bench.py cpu_baseline): mark every push-sum node active,
 * so a round costs what a steady-state round costs (every node sends) without the
 * activation pre-roll, which at P = 1e9 would take minutes of full-population
 * passes.  Not an SRS v1 transition -- never used by a parity check.  Returns the
 * number of nodes it activated, or -1 for gossip. */
int64_t or_activate_all(or_sim* s) {
    if (s->alg != OR_PUSHSUM) return -1;
    int64_t n = 0;
    for (int64_t i = 0; i < s->P; ++i) {
        n += !s->active[i];
        s->active[i] = 1;
    }
    return n;
}

int64_t or_active_count(const or_sim* s) {
    int64_t a = 0;
    for (int64_t i = 0; i < s->P; ++i) {
        if (s->alg == OR_GOSSIP) {
            int32_t ci = s->c[i];
            a += (i == s->seed_node || ci >= 1) && ci <= 10;
        } else {
            a += s->active[i];
        }
    }
    return a;
}

int or_read_state(const or_sim* s, int64_t first, int64_t count, int32_t* c,
                  double* sv, double* wv, uint8_t* flags) {
    if (first < 0 || count < 0 || first + count > s->P) return -1;
    for (int64_t q = 0; q < count; ++q) {
        int64_t i = first + q;
        if (s->alg == OR_GOSSIP) {
            int32_t ci = s->c[i];
            if (c) c[q] = ci;
            if (sv) sv[q] = 0.0;
            if (wv) wv[q] = 0.0;
            if (flags) {
                int act = (i == s->seed_node || ci >= 1) && ci <= 10;
                flags[q] = (uint8_t)(act | ((ci >= 11) << 1));
            }
        } else {
            if (c) c[q] = 0;
            if (sv) sv[q] = s->s[i];
            if (wv) wv[q] = s->w[i];
            if (flags) flags[q] = (uint8_t)(s->active[i] | (s->conv[i] << 1) | (s->cnt[i] << 2));
        }
    }
    return 0;
}

/* ---------------------------------------------------------------- sampled receivers */
/* One push-sum round r for a sample of receivers, from a full round-r state
 * supplied by the caller (e.g. read back from the HIP path): the same rules as
 * pushsum_round (SRS v1 B.4, restating MainPushSum, Program.fs:101-131), pulled
 * per receiver instead of pushed per sender, so that the product's round can be
 * checked at populations the whole-network oracle cannot hold (P = 1e9):
 *   - every lattice neighbour n of receiver j (j's slot order, Program.fs:246-257)
 *     sends to j iff it is active with degree > 0 and its round-r draw
 *     U_PUSHSUM(n, r, deg n) picks the slot whose target is j;
 *   - Imp3D random in-senders of j = every i with rnd[i] == j (Program.fs:258-260,
 *     rnd recomputed here from the TOPO stream, not taken from the product), each
 *     sending iff its draw picks its random slot; folded by ascending i;
 *   - own half, the fold, the ratio test and the flags as pushsum_round.
 * Inputs s, w, flags (bit0 active, bit1 converged, bits2-3 count) hold all P
 * nodes at the start of round r; ids are distinct receivers.  Outputs per id.
 * Returns the number of sampled receivers that converge in this round, or -1. */
int64_t or_pushsum_receivers(int topology, int64_t num_nodes, uint64_t seed, uint32_t round,
                             const double* sv, const double* wv, const uint8_t* flags,
                             const int64_t* ids, int64_t nids, double* s_out, double* w_out,
                             uint8_t* flags_out, int threads) {
    or_sim c;
    memset(&c, 0, sizeof c);
    int64_t P, T, g;
    if (or_resolve(num_nodes, topology, &P, &T, &g)) return -1;
    c.topo = topology; c.alg = OR_PUSHSUM; c.threads = threads; c.seed = seed;
    c.P = P; c.T = T; c.g = g;
    const int nt = nthreads(&c);
    int32_t* pos = (int32_t*)malloc(sizeof(int32_t) * P);
    int64_t* roff = (int64_t*)calloc(nids + 1, sizeof(int64_t));
    int64_t* rcur = (int64_t*)calloc(nids + 1, sizeof(int64_t));
    uint32_t* rsrc = NULL;
    if (!pos || !roff || !rcur) { free(pos); free(roff); free(rcur); return -1; }
    #pragma omp parallel for num_threads(nt) schedule(static)
    for (int64_t i = 0; i < P; ++i) pos[i] = -1;
    for (int64_t q = 0; q < nids; ++q) {
        if (ids[q] < 0 || ids[q] >= P || pos[ids[q]] >= 0) { free(pos); free(roff); free(rcur); return -1; }
        pos[ids[q]] = (int32_t)q;
    }
    if (topology == OR_FULL) {
        /* full topology (Program.fs:209-216): every active sender's round-r target,
         * t = U(P-1) mapped past i (as pushsum_round_full); senders of the sampled
         * receivers grouped per receiver, then sorted below */
        c.rnd = (uint32_t*)malloc(sizeof(uint32_t) * P);
        if (!c.rnd) { free(pos); free(roff); free(rcur); return -1; }
        #pragma omp parallel for num_threads(nt) schedule(static)
        for (int64_t i = 0; i < P; ++i) {
            uint32_t t = NONE_U32;
            if ((flags[i] & 1) && P > 1) {
                const uint32_t k = or_uniform(seed, OR_STREAM_PUSHSUM, (uint64_t)i, round, (uint32_t)(P - 1));
                t = (int64_t)k < i ? k : (uint32_t)(k + 1);
            }
            c.rnd[i] = t;
        }
    } else if (topology == OR_IMP3D) {
        c.rnd = (uint32_t*)malloc(sizeof(uint32_t) * P);
        if (!c.rnd) { free(pos); free(roff); free(rcur); return -1; }
        #pragma omp parallel for num_threads(nt) schedule(static)
        for (int64_t i = 0; i < P; ++i)
            c.rnd[i] = or_uniform(seed, OR_STREAM_TOPO, (uint64_t)i, 0, (uint32_t)(P - 1));
    }
    if (topology == OR_IMP3D || topology == OR_FULL) {
        /* random in-senders of the sampled receivers, grouped per receiver */
        #pragma omp parallel for num_threads(nt) schedule(static)
        for (int64_t i = 0; i < P; ++i) {
            int32_t q = c.rnd[i] == NONE_U32 ? -1 : pos[c.rnd[i]];
            if (q >= 0) {
                #pragma omp atomic
                roff[q + 1] += 1;
            }
        }
        for (int64_t q = 0; q < nids; ++q) roff[q + 1] += roff[q];
        memcpy(rcur, roff, sizeof(int64_t) * (nids + 1));
        rsrc = (uint32_t*)malloc(sizeof(uint32_t) * (roff[nids] + 1));
        if (!rsrc) { free(c.rnd); free(pos); free(roff); free(rcur); return -1; }
        #pragma omp parallel for num_threads(nt) schedule(static)
        for (int64_t i = 0; i < P; ++i) {
            int32_t q = c.rnd[i] == NONE_U32 ? -1 : pos[c.rnd[i]];
            if (q >= 0) {
                int64_t at;
                #pragma omp atomic capture
                at = rcur[q]++;
                rsrc[at] = (uint32_t)i;
            }
        }
    }
    int64_t alerts = 0;
    #pragma omp parallel for num_threads(nt) schedule(dynamic, 256) reduction(+ : alerts)
    for (int64_t q = 0; q < nids; ++q) {
        const int64_t j = ids[q];
        const uint8_t fj = flags[j];
        int active = fj & 1, conv = (fj >> 1) & 1, cnt = (fj >> 2) & 3;
        const int halve = active && degree(&c, j) > 0;
        double acc_s = halve ? sv[j] * 0.5 : sv[j];
        double acc_w = halve ? wv[j] * 0.5 : wv[j];
        int recv = 0;
        /* lattice senders in j's slot order (none on the full topology) */
        int64_t nb[7];
        const int d = topology == OR_FULL ? 0 : topology == OR_LINE ? line_nbrs(P, j, nb) : lattice_nbrs(g, j, nb);
        for (int k = 0; k < d; ++k) {
            const int64_t n = nb[k];
            if (!(flags[n] & 1)) continue;
            const int64_t dn = degree(&c, n);
            if (dn <= 0) continue;
            int rnd_slot;
            const uint32_t kk = or_uniform(seed, OR_STREAM_PUSHSUM, (uint64_t)n, round, (uint32_t)dn);
            if (slot_target(&c, n, kk, &rnd_slot) != j || rnd_slot) continue;
            acc_s = acc_s + sv[n] * 0.5;
            acc_w = acc_w + wv[n] * 0.5;
            recv = 1;
        }
        /* random in-senders (full: every sender) by ascending id */
        if (topology == OR_IMP3D || topology == OR_FULL) {
            const int64_t b = roff[q], e = roff[q + 1];
            for (int64_t p = b + 1; p < e; ++p) { /* insertion sort: a handful per receiver */
                uint32_t v = rsrc[p];
                int64_t t = p;
                while (t > b && rsrc[t - 1] > v) { rsrc[t] = rsrc[t - 1]; --t; }
                rsrc[t] = v;
            }
            for (int64_t p = b; p < e; ++p) {
                const int64_t i = rsrc[p];
                if (!(flags[i] & 1)) continue;
                if (topology == OR_IMP3D) {
                    const int64_t di = degree(&c, i);
                    const uint32_t kk = or_uniform(seed, OR_STREAM_PUSHSUM, (uint64_t)i, round, (uint32_t)di);
                    if (kk != (uint32_t)(di - 1)) continue; /* the random slot is the last one */
                } /* (full: rsrc holds exactly this round's senders to j) */
                acc_s = acc_s + sv[i] * 0.5;
                acc_w = acc_w + wv[i] * 0.5;
                recv = 1;
            }
        }
        if (recv) {
            if (!conv) {
                const double r_old = sv[j] / wv[j];
                const double r_new = acc_s / acc_w;
                cnt = (fabs(r_new - r_old) > 1e-10) ? 0 : cnt + 1;
                if (cnt == 3) { conv = 1; alerts += 1; }
            }
            active = 1;
        }
        s_out[q] = acc_s;
        w_out[q] = acc_w;
        flags_out[q] = (uint8_t)(active | (conv << 1) | ((cnt & 3) << 2));
    }
    free(rsrc); free(c.rnd); free(pos); free(roff); free(rcur);
    return alerts;
}
