// gossip_cli.cpp -- command-line front-end with the reference's surface:
//
//   gossip <num_nodes> <topology> <algorithm> [--seed S] [--max-rounds R]
//          [--device D] [--stats]
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
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/gossip_hip.h"

static int usage() {
    std::fprintf(stderr,
                 "usage: gossip <num_nodes> <line|full|3D|Imp3D> <gossip|push-sum> "
                 "[--seed S] [--max-rounds R] [--device D] [--stats]\n");
    return 2;
}

int main(int argc, char** argv) {
    if (argc < 4) return usage();
    gp_config cfg;
    std::memset(&cfg, 0, sizeof cfg);
    char* end = nullptr;
    cfg.num_nodes = std::strtoll(argv[1], &end, 10);
    if (!end || *end) {
        std::fprintf(stderr, "num_nodes must be an integer: '%s'\n", argv[1]);
        return 2;
    }
    cfg.seed = 1;
    cfg.num_gpus = 1;
    bool stats = false;
    if (const char* e = std::getenv("GOSSIP_SEED")) cfg.seed = std::strtoull(e, nullptr, 10);
    for (int i = 4; i < argc; ++i) {
        std::string a = argv[i];
        if (a == "--seed" && i + 1 < argc) cfg.seed = std::strtoull(argv[++i], nullptr, 10);
        else if (a == "--max-rounds" && i + 1 < argc) cfg.max_rounds = std::strtoll(argv[++i], nullptr, 10);
        else if (a == "--device" && i + 1 < argc) cfg.device = std::atoi(argv[++i]);
        else if (a == "--stats") stats = true;
        else return usage();
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
    cfg.topology = topo;
    cfg.algorithm = alg;

    gp_sim* sim = nullptr;
    int rc = gp_create(&cfg, &sim);
    if (rc) {
        std::fprintf(stderr, "gp_create failed (%d): %s\n", rc, gp_last_error());
        return 1;
    }
    std::printf(alg == GP_GOSSIP ? "Gossip Starts\n" : "Push Sum Starts\n");
    std::fflush(stdout);
    gp_result res;
    rc = gp_run(sim, &res);
    if (rc) {
        std::fprintf(stderr, "gp_run failed (%d): %s\n", rc, gp_last_error());
        gp_destroy(sim);
        return 1;
    }
    int code = 0;
    if (res.status == GP_STATUS_CONVERGED) {
        std::printf("Convergence Time: %f ms\n", res.elapsed_ms);
    } else {
        std::printf("Not converged after %lld rounds (%lld of %lld alerts)\n", (long long)res.rounds,
                    (long long)res.converged, (long long)res.threshold);
        code = 3;
    }
    if (stats) {
        std::printf("rounds=%lld population=%lld threshold=%lld node_updates_per_s=%.4e alg_hbm_GBps=%.1f\n",
                    (long long)res.rounds, (long long)res.population, (long long)res.threshold,
                    res.node_updates_per_s, res.elapsed_ms > 0 ? res.hbm_bytes_alg / (res.elapsed_ms * 1e6) : 0.0);
    }
    gp_destroy(sim);
    return code;
}
