/*
 * gossip_hip.h -- C-ABI of libgossip_hip.so, the MI355X-native replacement for
 * the gossip / push-sum hot path of sharwarimarathe/GossipProtocol.
 *
 * The reference has no plugin or operator API: its only caller of the path is
 * `main` in /root/reference/Project2/Program.fs (cited below as Program.fs:N),
 * driven by the CLI `dotnet run <num_nodes> <topology> <algorithm>`
 * (README.md:1, argv parse Program.fs:32-34).  Each entry point below names the
 * block of Program.fs it replaces; a front-end keeps the argv/stdout contract
 * and binds these symbols (F# P/Invoke stub: INTEGRATION.md).
 *
 * Conventions: plain C types and blittable structs only (no torch or HIP
 * types), return 0 on success or a negative GP_E* code; gp_last_error() holds
 * the message for the calling thread.  The library owns all device memory and
 * streams; the caller owns cfg/out/readback buffers.  A gp_sim is not
 * reentrant: one caller thread per handle.
 *
 * Semantics: the synchronous-round specification SRS v1 (SURVEY.md Appendix
 * B).  Randomness is Philox4x32-10 keyed by cfg.seed, so runs are
 * reproducible and bit-identical to the CPU oracle.
 */
#ifndef GOSSIP_HIP_H
#define GOSSIP_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GP_VERSION 10100 /* 1.1.0 */
/* Largest population (node ids are 32-bit; tiles of 1024 ids must not wrap). */
#define GP_MAX_POPULATION 0xFFFFF000u

/* topology strings "line" | "full" | "3D" | "Imp3D" (Program.fs:180,209,238,258) */
enum { GP_LINE = 0, GP_FULL = 1, GP_3D = 2, GP_IMP3D = 3 };
/* algorithm strings "gossip" | "push-sum" (Program.fs:196,202) */
enum { GP_GOSSIP = 0, GP_PUSHSUM = 1 };
/* gp_result.status */
enum { GP_STATUS_CONVERGED = 0, GP_STATUS_MAX_ROUNDS = 1, GP_STATUS_RUNNING = 2 };
/* error codes */
enum {
    GP_OK = 0,
    GP_EINVAL = -1,    /* bad argument / unknown topology or algorithm */
    GP_ENOMEM = -2,    /* host or device allocation failed */
    GP_EHIP = -3,      /* HIP runtime error */
    GP_ENCCL = -4,     /* RCCL error */
    GP_ESTATE = -5,    /* call not valid in the handle's state */
    GP_ENODEV = -6     /* no usable gfx950 device */
};
/* gp_config.flags */
enum {
    GP_FLAG_KERNEL_TIMING = 1, /* bracket every round kernel with HIP events (gp_kernel_stats) */
    GP_FLAG_VIRTUAL_RANKS = 2  /* num_gpus > 1 slabs in this process on `device` (the multi-GPU
                                  exchange with device copies instead of RCCL; for testing) */
};

typedef struct gp_sim gp_sim;

/* Replaces Program.fs:32-34 (argv) plus the constants the reference hard-codes. */
typedef struct gp_config {
    int64_t num_nodes;   /* argv[0]: `nodes` (Program.fs:32) */
    int32_t topology;    /* GP_LINE .. GP_IMP3D (argv[1], Program.fs:33) */
    int32_t algorithm;   /* GP_GOSSIP | GP_PUSHSUM (argv[2], Program.fs:34) */
    uint64_t seed;       /* Philox key; replaces `new Random()` (Program.fs:86 et al.) */
    int32_t num_gpus;    /* 1; multi-GPU runs one process per GPU (gp_create_rank; launchers:
                            `gossip --gpus N` / GOSSIP_GPUS, bench.py --gpus N), or num_gpus
                            in-process slabs with GP_FLAG_VIRTUAL_RANKS */
    int32_t device;      /* HIP device ordinal for num_gpus == 1 */
    int64_t max_rounds;  /* cap; <= 0 means unlimited (the reference blocks forever, Program.fs:282) */
    int32_t flags;       /* GP_FLAG_* */
    int32_t reserved;
} gp_config;

/* What the scheduler actor reports (Program.fs:53-55) plus throughput. */
typedef struct gp_result {
    int64_t rounds;             /* rounds executed by this handle so far */
    int64_t converged;          /* cumulative alerts (scheduler `counter`, Program.fs:52) */
    int64_t population;         /* P: nodes simulated */
    int64_t threshold;          /* T: alerts needed (Program.fs:53) */
    double elapsed_ms;          /* round-loop wall time of this call (Stopwatch, Program.fs:35,194,54) */
    double node_updates_per_s;  /* P * rounds / elapsed */
    double hbm_bytes_alg;       /* algorithmic HBM bytes of the rounds run */
    int32_t status;             /* GP_STATUS_* */
    int32_t reserved;
} gp_result;

typedef struct gp_info {
    int64_t population, threshold, grid;  /* P, T, g (g = 0 for line/full) */
    int64_t seed_node;                    /* `choice` (Program.fs:193,221,263) */
    int64_t rounds, alerts_total, active; /* progress */
    int32_t topology, algorithm;
    int32_t device, num_gpus;             /* num_gpus = ranks sharing the population */
    int64_t slab_first, slab_count;       /* node ids owned by this handle */
} gp_info;

/* Library version (GP_VERSION). */
int gp_version(void);
/* Message for the last failing call on this thread ("" if none). */
const char* gp_last_error(void);

/* CLI helpers: parse the reference's case-sensitive strings (Program.fs:178-279);
 * "imp3D" is accepted as an alias of "Imp3D".  Return the enum or GP_EINVAL. */
int gp_parse_topology(const char* s);
int gp_parse_algorithm(const char* s);
/* Resolve P (population), T (alert threshold) and g (grid edge) for n nodes:
 * line/full P = n+1, T = n (Program.fs:170-171,53); 3D/Imp3D g = ceil(cbrt n)
 * exactly, P = T = g^3 (Program.fs:239-240). */
int gp_resolve(int64_t num_nodes, int32_t topology, int64_t* P, int64_t* T, int64_t* g);

/* Replaces Program.fs:36-39,63,65-176 and the topology blocks 180-191 / 209-216 /
 * 238-261: allocates the SoA node state on the device, builds the implicit
 * topology (Imp3D: random edges + receiver-sorted in-lists), initialises
 * s = id, w = 1, count = 1, rumours = 0, and picks the seed node. */
int gp_create(const gp_config* cfg, gp_sim** out);

/* Multi-GPU: one process per GPU.  `unique_id` is the 128-byte RCCL id from
 * gp_get_unique_id() on rank 0, broadcast by the caller.  Nodes are split into
 * contiguous id slabs (plane-aligned for 3D/Imp3D). */
int gp_get_unique_id(uint8_t unique_id[128]);
int gp_create_rank(const gp_config* cfg, int32_t rank, int32_t world, const uint8_t unique_id[128],
                   gp_sim** out);

/* Launcher rendezvous without a host framework (gossip --gpus N, bench.py
 * --gpus N, the F# front-end): the launcher starts one process per GPU before
 * any of them touches a GPU and hands all of them one fresh file path.  Rank 0
 * calls gp_get_unique_id and publishes the 128 bytes at `path` (written under a
 * private name, then renamed, so a reader never sees a partial id); every other
 * rank waits for the file (at most timeout_ms; < 0 waits forever) and reads it.
 * Then every rank calls gp_create_rank with the same id.  The launcher removes
 * the file afterwards.  The path must be fresh: rank 0 fails with GP_ESTATE when
 * a file is already there.  If GOSSIP_RDV_NONCE is set in the environment (the
 * launchers set one value per launch), rank 0 appends it to the id and readers
 * accept only a file carrying the same nonce, so a file left at a reused path by
 * a crashed run is never taken for this run's id. */
int gp_rendezvous_id(int32_t rank, const char* path, int32_t timeout_ms, uint8_t unique_id[128]);

/* Replaces the message loop Program.fs:84-131,141-163 plus the scheduler
 * Program.fs:41-61: runs synchronous rounds until the cumulative alert count
 * reaches T (then status = GP_STATUS_CONVERGED) or max_rounds is hit. */
int gp_run(gp_sim* sim, gp_result* out);

/* Runs at most `nrounds` rounds (stops after the converging round).  Writes the
 * per-round alert counts of the executed rounds to alerts_per_round_out (may be
 * NULL).  Returns the number of rounds executed (>= 0) or a GP_E* code. */
int64_t gp_step(gp_sim* sim, int64_t nrounds, int64_t* alerts_per_round_out);

/* Copies node state [first, first+count) to caller buffers; null pointers are
 * skipped.  c: gossip rumour counters (push-sum: 0).  s, w: push-sum sum and
 * weight (gossip: 0).  flags: bit0 active, bit1 converged, bits2-3 push-sum
 * stability count.  In multi-GPU mode the range must lie in this rank's slab. */
int gp_read_state(gp_sim* sim, int64_t first, int64_t count, int32_t* c, double* s, double* w,
                  uint8_t* flags);

/* Neighbour list of node i in the reference's slot order (Program.fs:182-191,
 * 211-216, 246-260).  Writes min(deg, cap) ids; returns deg or a GP_E* code. */
int gp_neighbors(gp_sim* sim, int64_t node, int64_t* out, int64_t cap);

int gp_get_info(gp_sim* sim, gp_info* out);
/* Blocks until all work queued by the handle has finished. */
int gp_sync(gp_sim* sim);
/* Round-kernel timing (GP_FLAG_KERNEL_TIMING): sum of HIP-event durations of the
 * dominant per-round kernel and the number of launches measured since the last
 * reset; `name` receives the kernel's name (may be NULL). */
int gp_kernel_stats(gp_sim* sim, double* total_ms, int64_t* launches, char* name, int32_t name_cap,
                    int32_t reset);
/* Algorithmic HBM bytes per node-round of the dominant kernel for the current
 * state. */
double gp_alg_bytes_per_node(gp_sim* sim);

void gp_destroy(gp_sim* sim);

#ifdef __cplusplus
}
#endif
#endif /* GOSSIP_HIP_H */
