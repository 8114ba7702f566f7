/*
 * srs_oracle.h -- CPU oracle for the synchronous-round restatement (SRS v1) of
 * the reference's gossip / push-sum hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * or the timed CPU baseline.  The product (gossipprotocol_amd / libgossip_hip)
 * never links or calls it.
 *
 * Parity status: the reference (/root/reference/Project2/Program.fs) is an
 * asynchronous Akka.NET program with `new Random()` per draw and ships no
 * tests, fixtures or golden vectors.  End-to-end parity
 * with the reference is therefore "parity unpinned".  What IS pinned:
 *   - Philox4x32-10 against the Random123 known-answer vectors;
 *   - neighbour orders against a literal transliteration of Program.fs:180-261;
 *   - every simulation rule against the SRS v1 text,
 *     cross-checked by an independent pure-Python restatement (srs_py.py).
 *
 * Formulation: "push" -- each sender computes its target and an ordering key,
 * messages are bucketed per receiver and folded in key order.  This is
 * deliberately a different formulation from the HIP kernels (which pull).
 */
#ifndef SRS_ORACLE_H
#define SRS_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { OR_LINE = 0, OR_FULL = 1, OR_3D = 2, OR_IMP3D = 3 };
enum { OR_GOSSIP = 0, OR_PUSHSUM = 1 };
enum { OR_STREAM_TOPO = 0, OR_STREAM_START = 1, OR_STREAM_GOSSIP = 2,
       OR_STREAM_PUSHSUM = 3, OR_STREAM_INJECT = 4 };

typedef struct or_sim or_sim;

/* Philox4x32-10 (Random123).  ctr[4], key[2] -> out[4]. */
void or_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
/* U(m) = floor(((y<<32)|x) * m / 2^64), x,y = first two Philox words. */
uint32_t or_uniform(uint64_t seed, uint32_t stream, uint64_t node, uint32_t round, uint32_t m);
/* smallest g >= 0 with g^3 >= n */
int64_t or_icbrt_ceil(int64_t n);
/* population / threshold / grid for (n, topology); returns 0 or -1 on bad input */
int or_resolve(int64_t n, int topology, int64_t* P, int64_t* T, int64_t* g);

or_sim* or_create(int64_t num_nodes, int topology, int algorithm, uint64_t seed,
                  int64_t max_rounds, int threads);
void or_destroy(or_sim* s);
/* Run up to nrounds rounds; stops after the round in which cumulative alerts
 * reach T.  alerts_out (may be NULL) receives one entry per executed round.
 * Returns rounds executed (>= 0). */
int64_t or_step(or_sim* s, int64_t nrounds, int64_t* alerts_out);
int64_t or_rounds_done(const or_sim* s);
int64_t or_alerts_total(const or_sim* s);
int64_t or_population(const or_sim* s);
int64_t or_threshold(const or_sim* s);
int64_t or_seed_node(const or_sim* s);
int64_t or_active_count(const or_sim* s);
/* bench.py cpu_baseline timing only: every push-sum node active (not an SRS v1 transition) */
int64_t or_activate_all(or_sim* s);
/* neighbour list of node i in reference slot order; returns degree.
 * out may be NULL (degree only). */
int or_neighbors(const or_sim* s, int64_t i, int64_t* out);
/* Copy state [first, first+count) -- null pointers skipped.  flags: bit0
 * active, bit1 converged, bits2-3 push-sum stability count. */
int or_read_state(const or_sim* s, int64_t first, int64_t count, int32_t* c,
                  double* sv, double* wv, uint8_t* flags);

/* Push-sum round `round` for the distinct receivers ids[0..nids) from a full
 * round-start state (all P nodes: s, w, flags as or_read_state) -- the check of
 * the product's round at populations the whole-network oracle cannot run.
 * Returns how many sampled receivers converge in the round, -1 on bad input. */
int64_t or_pushsum_receivers(int topology, int64_t num_nodes, uint64_t seed, uint32_t round,
                             const double* sv, const double* wv, const uint8_t* flags,
                             const int64_t* ids, int64_t nids, double* s_out, double* w_out,
                             uint8_t* flags_out, int threads);

#ifdef __cplusplus
}
#endif
#endif
