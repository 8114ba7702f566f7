/// Drop-in front-end: `dotnet run <num_nodes> <topology> <algorithm>` with the
/// reference's argv (Program.fs:32-34 of sharwarimarathe/GossipProtocol) and
/// stdout contract ("Gossip Starts" / "Push Sum Starts", then
/// "Convergence Time: %f ms"), running the synchronous rounds on an MI355X
/// through libgossip_hip.so.  UNVERIFIED here (no .NET SDK in the image); the
/// C++ build of the same front-end is gossipprotocol_amd/csrc/gossip_cli.cpp.
module Program

open System
open GossipHip

[<EntryPoint>]
let main argv =
    if argv.Length < 3 then
        eprintfn "usage: dotnet run <num_nodes> <line|full|3D|Imp3D> <gossip|push-sum>"
        2
    else
        let topo = gp_parse_topology argv.[1]
        let alg = gp_parse_algorithm argv.[2]
        if alg < 0 then
            printfn "option invalid"
            2
        elif topo < 0 then
            eprintfn "%s" (lastError ())
            2
        else
            let mutable cfg = GpConfig()
            cfg.NumNodes <- int64 argv.[0]
            cfg.Topology <- topo
            cfg.Algorithm <- alg
            cfg.Seed <- (match Environment.GetEnvironmentVariable "GOSSIP_SEED" with
                         | null -> 1UL
                         | s -> uint64 s)
            cfg.NumGpus <- 1
            let mutable sim = 0n
            let rc = gp_create(&cfg, &sim)
            if rc <> 0 then
                eprintfn "gp_create failed (%d): %s" rc (lastError ())
                1
            else
                printfn (if alg = 0 then "Gossip Starts" else "Push Sum Starts")
                let mutable res = GpResult()
                let rc = gp_run(sim, &res)
                gp_destroy sim
                if rc <> 0 then
                    eprintfn "gp_run failed (%d): %s" rc (lastError ())
                    1
                elif res.Status = 0 then
                    printfn "Convergence Time: %f ms" res.ElapsedMs
                    0
                else
                    printfn "Not converged after %d rounds" res.Rounds
                    3
