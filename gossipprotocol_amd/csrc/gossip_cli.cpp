// gossip_cli.cpp -- command-line front-end with the reference's surface:
//
//   gossip <num_nodes> <topology> <algorithm> [--seed S] [--max-rounds R]
//          [--gpus G] [--device D] [--stats]
//
// mirrors `dotnet run num_nodes topology algorithm` (README.md:1, argv parse
// Program.fs:32-34) and its stdout contract: "Gossip Starts" / "Push Sum Starts"
// (Program.fs:198,203) then "Convergence Time: %f ms" (Program.fs:55), exit 0
// (Environment.Exit(0), Program.fs:56).  An unknown algorithm prints
// "option invalid" (Program.fs:207) and, unlike the reference (which then
// blocks on ReadKey, Program.fs:282), exits 2; an unknown topology (silently
// ignored by Program.fs:279) is reported and exits 2.
//
// The timed region matches the reference's Stopwatch: it starts after the
// topology build (Program.fs:194,219,264) and stops at the T-th alert
// (Program.fs:53-54).  The F# front-end in fsharp/ is the same program over
// P/Invoke; this one is the C++ build of it for hosts without a .NET SDK.
//
// Several GPUs (--gpus G, or GOSSIP_GPUS=G): this process is the
// launcher.  It never calls into HIP or RCCL; it forks one rank process per GPU
// first, and every rank joins through gp_rendezvous_id (rank 0's RCCL id in a
// fresh file) + gp_create_rank on device `rank`.  Rank 0 prints the stdout
// contract; the launcher waits for all ranks, and if one fails it stops the
// others and exits non-zero -- a multi-GPU request never falls back to one GPU.
// `--device D` with G > 1 is the one-GPU rehearsal: every rank on device D,
// each with its own RCCL host id (RCCL's socket transport on loopback), for
// boxes with a single MI355X.
#include <cerrno>
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <sys/stat.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <unistd.h>

#include "../../include/gossip_hip.h"

namespace {

int usage() {
    std::fprintf(stderr,
                 "usage: gossip <num_nodes> <line|full|3D|Imp3D> <gossip|push-sum> "
                 "[--seed S] [--max-rounds R] [--gpus G] [--device D] [--stats]\n");
    return 2;
}

struct Args {
    gp_config cfg;
    int gpus = 1;
    bool device_set = false;  // --device given: with gpus > 1, every rank on that device
    bool stats = false;
};

// Run this process's share: the whole network (world 1) or rank `rank` of
// `world`.  Only rank 0 writes the stdout contract.  Returns the exit code.
int run(const Args& a, int rank, int world, const char* rdv) {
    gp_config cfg = a.cfg;
    gp_sim* sim = nullptr;
    int rc;
    if (world == 1) {
        rc = gp_create(&cfg, &sim);
    } else {
        uint8_t uid[128];
        if ((rc = gp_rendezvous_id(rank, rdv, 600000, uid)) == 0) {
            cfg.num_gpus = world;
            if (!a.device_set) cfg.device = rank;
            // RCCL prints its version line on stdout when the communicator starts: keep
            // stdout for the reference's contract (the line goes to stderr)
            std::fflush(stdout);
            const int saved = dup(1);
            if (saved >= 0) dup2(2, 1);
            rc = gp_create_rank(&cfg, rank, world, uid, &sim);
            std::fflush(stdout);
            if (saved >= 0) {
                dup2(saved, 1);
                close(saved);
            }
        }
    }
    if (rc) {
        std::fprintf(stderr, "[rank %d/%d] gp_create failed (%d): %s\n", rank, world, rc, gp_last_error());
        return 1;
    }
    const bool lead = rank == 0;
    if (lead) {
        std::printf(cfg.algorithm == GP_GOSSIP ? "Gossip Starts\n" : "Push Sum Starts\n");
        std::fflush(stdout);
    }
    gp_result res;
    rc = gp_run(sim, &res);
    if (rc) {
        std::fprintf(stderr, "[rank %d/%d] gp_run failed (%d): %s\n", rank, world, rc, gp_last_error());
        gp_destroy(sim);
        return 1;
    }
    int code = 0;
    if (res.status != GP_STATUS_CONVERGED) code = 3;
    if (lead) {
        if (code == 0)
            std::printf("Convergence Time: %f ms\n", res.elapsed_ms);
        else
            std::printf("Not converged after %lld rounds (%lld of %lld alerts)\n", (long long)res.rounds,
                        (long long)res.converged, (long long)res.threshold);
        if (a.stats)
            std::printf("rounds=%lld population=%lld threshold=%lld gpus=%d node_updates_per_s=%.4e "
                        "alg_hbm_GBps=%.1f\n",
                        (long long)res.rounds, (long long)res.population, (long long)res.threshold, world,
                        res.node_updates_per_s,  // whole network: P * rounds / elapsed
                        res.elapsed_ms > 0 ? res.hbm_bytes_alg / (res.elapsed_ms * 1e6) : 0.0);
        std::fflush(stdout);
    }
    gp_destroy(sim);
    return code;
}

// Fork `world` rank processes, wait for all of them; the first failure stops
// the rest (SIGTERM, then SIGKILL) and becomes the exit code.
int launch(const Args& a) {
    const int world = a.gpus;
    const char* tmpdir = std::getenv("TMPDIR");
    std::string dir = std::string(tmpdir && *tmpdir ? tmpdir : "/tmp") + "/gossip_rdv_XXXXXX";
    if (!mkdtemp(&dir[0])) {
        std::fprintf(stderr, "gossip: mkdtemp(%s) failed: %s\n", dir.c_str(), std::strerror(errno));
        return 1;
    }
    const std::string rdv = dir + "/rccl_id";
    const pid_t launcher = getpid();
    // this launch's rendezvous nonce (gp_rendezvous_id): the ranks inherit it through fork
    const std::string nonce = std::to_string((long long)launcher) + "-" + dir.substr(dir.size() - 6);
    setenv("GOSSIP_RDV_NONCE", nonce.c_str(), 1);
    std::fflush(stdout);
    std::fflush(stderr);
    std::vector<pid_t> pids;
    for (int r = 0; r < world; ++r) {
        const pid_t p = fork();
        if (p < 0) {
            std::fprintf(stderr, "gossip: fork failed: %s\n", std::strerror(errno));
            for (pid_t q : pids) kill(q, SIGKILL);
            for (pid_t q : pids) waitpid(q, nullptr, 0);
            rmdir(dir.c_str());
            return 1;
        }
        if (p == 0) {  // rank process: nothing has touched a GPU yet
            if (a.device_set) {  // one-GPU rehearsal: distinct RCCL host ids -> socket transport
                const std::string host = "gossip-rehearsal-" + std::to_string((long long)launcher) + "-" + std::to_string(r);
                setenv("NCCL_HOSTID", host.c_str(), 1);
                setenv("NCCL_SOCKET_IFNAME", "lo", 0);
                setenv("NCCL_IB_DISABLE", "1", 0);
            }
            const int code = run(a, r, world, rdv.c_str());
            std::fflush(stdout);
            std::fflush(stderr);
            _exit(code);
        }
        pids.push_back(p);
    }
    int result = 0, lead = -1;
    bool stopping = false;
    size_t live = pids.size();
    while (live > 0) {
        int st = 0;
        const pid_t p = waitpid(-1, &st, 0);
        if (p < 0) {
            if (errno == EINTR) continue;
            break;
        }
        int r = -1;
        for (size_t k = 0; k < pids.size(); ++k)
            if (pids[k] == p) r = (int)k;
        if (r < 0) continue;
        pids[r] = -1;
        --live;
        const int code = WIFEXITED(st) ? WEXITSTATUS(st) : 128 + (WIFSIGNALED(st) ? WTERMSIG(st) : 0);
        if (r == 0) lead = code;
        if (code != 0 && code != 3 && !stopping) {
            std::fprintf(stderr, "gossip: rank %d of %d failed (exit %d); stopping the other ranks\n", r, world, code);
            result = code;
            stopping = true;
            for (pid_t q : pids)
                if (q > 0) kill(q, SIGTERM);
            // give them a moment, then make sure
            for (int t = 0; t < 50 && live > 0; ++t) {
                int st2 = 0;
                const pid_t p2 = waitpid(-1, &st2, WNOHANG);
                if (p2 > 0) {
                    for (auto& q : pids)
                        if (q == p2) {
                            q = -1;
                            --live;
                        }
                } else {
                    usleep(100000);
                }
            }
            for (pid_t q : pids)
                if (q > 0) kill(q, SIGKILL);
        }
    }
    unlink(rdv.c_str());
    rmdir(dir.c_str());
    if (result) return result;
    return lead < 0 ? 1 : lead;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 4) return usage();
    Args a;
    std::memset(&a.cfg, 0, sizeof a.cfg);
    char* end = nullptr;
    a.cfg.num_nodes = std::strtoll(argv[1], &end, 10);
    if (!end || *end) {
        std::fprintf(stderr, "num_nodes must be an integer: '%s'\n", argv[1]);
        return 2;
    }
    a.cfg.seed = 1;
    a.cfg.num_gpus = 1;
    if (const char* e = std::getenv("GOSSIP_SEED")) a.cfg.seed = std::strtoull(e, nullptr, 10);
    if (const char* e = std::getenv("GOSSIP_GPUS")) a.gpus = std::atoi(e);
    for (int i = 4; i < argc; ++i) {
        std::string s = argv[i];
        if (s == "--seed" && i + 1 < argc) a.cfg.seed = std::strtoull(argv[++i], nullptr, 10);
        else if (s == "--max-rounds" && i + 1 < argc) a.cfg.max_rounds = std::strtoll(argv[++i], nullptr, 10);
        else if (s == "--device" && i + 1 < argc) {
            a.cfg.device = std::atoi(argv[++i]);
            a.device_set = true;
        } else if (s == "--gpus" && i + 1 < argc) a.gpus = std::atoi(argv[++i]);
        else if (s == "--stats") a.stats = true;
        else return usage();
    }
    if (a.gpus < 1) {
        std::fprintf(stderr, "--gpus / GOSSIP_GPUS must be >= 1 (got %d)\n", a.gpus);
        return 2;
    }
    const int topo = gp_parse_topology(argv[2]);
    if (topo < 0) {
        std::fprintf(stderr, "%s\n", gp_last_error());
        return 2;
    }
    const int alg = gp_parse_algorithm(argv[3]);
    if (alg < 0) {
        std::printf("option invalid\n");
        return 2;
    }
    a.cfg.topology = topo;
    a.cfg.algorithm = alg;
    if (a.gpus == 1) return run(a, 0, 1, nullptr);
    return launch(a);
}
