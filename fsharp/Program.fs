/// Drop-in front-end: `dotnet run <num_nodes> <topology> <algorithm>` with the
/// reference's argv (Program.fs:32-34 of sharwarimarathe/GossipProtocol) and
/// stdout contract ("Gossip Starts" / "Push Sum Starts", then
/// "Convergence Time: %f ms"), running the synchronous rounds on an MI355X
/// through libgossip_hip.so.
///
/// Optional fourth argument:
///   --sync-ref  run the F# synchronous-round reference (SyncRef.fs) instead;
///   --check     run SyncRef and libgossip_hip in lock step: per-round alerts and
///               the final node state must be identical (exit 4 otherwise).
/// UNVERIFIED here (no .NET SDK in the image); the C++ build of the same
/// front-end is gossipprotocol_amd/csrc/gossip_cli.cpp.
module Program

open System
open System.Diagnostics
open GossipHip

let private seedFromEnv () =
    match Environment.GetEnvironmentVariable "GOSSIP_SEED" with
    | null -> 1UL
    | s -> uint64 s

let private starts alg = if alg = 0 then "Gossip Starts" else "Push Sum Starts"

/// The F# reference alone: same stdout contract, wall time of the round loop.
let private runSyncRef (n: int64) topo alg seed =
    let sim = SyncRef.create n topo alg seed
    printfn "%s" (starts (int alg))
    let sw = Stopwatch.StartNew()
    while not sim.Done do
        SyncRef.step sim 1024 |> ignore
    sw.Stop()
    printfn "Convergence Time: %f ms" sw.Elapsed.TotalMilliseconds
    printfn "Rounds: %d" sim.Round
    0

/// SyncRef against libgossip_hip, round by round.
let private check (n: int64) topo alg seed =
    let mutable cfg = GpConfig()
    cfg.NumNodes <- n
    cfg.Topology <- int topo
    cfg.Algorithm <- int alg
    cfg.Seed <- seed
    cfg.NumGpus <- 1
    let mutable h = 0n
    let rc = gp_create (&cfg, &h)
    if rc <> 0 then
        eprintfn "gp_create failed (%d): %s" rc (lastError ())
        1
    else
        let ref = SyncRef.create n topo alg seed
        let buf = Array.zeroCreate<int64> 256
        let mutable ok = true
        let mutable rounds = 0
        while ok && not ref.Done do
            let got = int (gp_step (h, 256L, buf))
            let want = SyncRef.step ref 256
            if got <> want.Length || Array.sub buf 0 got <> want then
                eprintfn "alerts differ in rounds %d..%d" rounds (rounds + want.Length)
                ok <- false
            rounds <- rounds + want.Length
        let P = ref.Net.P
        let c, s, w, f = Array.zeroCreate<int32> P, Array.zeroCreate<float> P, Array.zeroCreate<float> P,
                         Array.zeroCreate<byte> P
        if ok && gp_read_state (h, 0L, int64 P, c, s, w, f) = 0 then
            let rc, rs, rw, rf = SyncRef.state ref
            // bit-exact: the same fold order and -ffp-contract=off arithmetic
            let sameF (a: float[]) (b: float[]) =
                Array.forall2 (fun (x: float) (y: float) -> BitConverter.DoubleToInt64Bits x = BitConverter.DoubleToInt64Bits y) a b
            if c <> rc || f <> rf || not (sameF s rs) || not (sameF w rw) then
                eprintfn "final state differs"
                ok <- false
        gp_destroy h
        if ok then
            printfn "SyncRef and libgossip_hip agree: %d rounds, %d alerts" rounds ref.AlertsTotal
            0
        else
            4

[<EntryPoint>]
let main argv =
    if argv.Length < 3 then
        eprintfn "usage: dotnet run <num_nodes> <line|full|3D|Imp3D> <gossip|push-sum> [--sync-ref|--check]"
        2
    else
        let mode = if argv.Length > 3 then argv.[3] else ""
        if mode = "--sync-ref" || mode = "--check" then
            match SyncRef.parseTopology argv.[1], SyncRef.parseAlgorithm argv.[2] with
            | _, None ->
                printfn "option invalid"
                2
            | None, _ ->
                eprintfn "unknown topology '%s' (line | full | 3D | Imp3D)" argv.[1]
                2
            | Some topo, Some alg ->
                if mode = "--sync-ref" then runSyncRef (int64 argv.[0]) topo alg (seedFromEnv ())
                else check (int64 argv.[0]) topo alg (seedFromEnv ())
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
            cfg.Seed <- seedFromEnv ()
            cfg.NumGpus <- 1
            let mutable sim = 0n
            let rc = gp_create (&cfg, &sim)
            if rc <> 0 then
                eprintfn "gp_create failed (%d): %s" rc (lastError ())
                1
            else
                printfn "%s" (starts alg)
                let mutable res = GpResult()
                let rc = gp_run (sim, &res)
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
