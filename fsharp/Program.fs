/// Drop-in front-end: `dotnet run <num_nodes> <topology> <algorithm>` with the
/// reference's argv (Program.fs:32-34 of sharwarimarathe/GossipProtocol) and
/// stdout contract ("Gossip Starts" / "Push Sum Starts", then
/// "Convergence Time: %f ms"), running the synchronous rounds on an MI355X
/// through libgossip_hip.so.
///
/// Options after the three positional arguments:
///   --sync-ref  run the F# synchronous-round reference (SyncRef.fs) instead;
///   --check     run SyncRef and libgossip_hip in lock step: per-round alerts and
///               the final node state must be identical (exit 4 otherwise);
///   --gpus G    (or GOSSIP_GPUS=G) one rank process per GPU: this process starts
///               G copies of itself before touching a GPU (GOSSIP_RANK /
///               GOSSIP_WORLD / GOSSIP_RDV in their environment), each joins
///               through gp_rendezvous_id + gp_create_rank on device `rank`, rank 0
///               prints; the first failing rank stops the others and sets the exit
///               code (the C++ CLI gossip_cli.cpp does the same with fork);
///   --device D  with --gpus: every rank on device D (one-GPU rehearsal, RCCL over
///               sockets: each rank gets its own NCCL_HOSTID).
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

/// Launcher side of --gpus: G rank processes of this program, waited for; the first
/// failure (exit code other than 0 / 3) stops the rest.
let private launchRanks (argv: string[]) (gpus: int) (rehearsal: bool) =
    let dir = IO.Path.Combine(IO.Path.GetTempPath(), "gossip_rdv_" + Guid.NewGuid().ToString("N"))
    IO.Directory.CreateDirectory dir |> ignore
    let rdv = IO.Path.Combine(dir, "rccl_id")
    // this program again: the apphost, or `dotnet <the assembly>` under dotnet run
    let host = Process.GetCurrentProcess().MainModule.FileName
    let pre = if IO.Path.GetFileNameWithoutExtension host = "dotnet" then [| Environment.GetCommandLineArgs().[0] |] else [||]
    let nonce = Guid.NewGuid().ToString("N")
    let procs =
        [| for r in 0 .. gpus - 1 ->
               let psi = ProcessStartInfo(host)
               for a in Array.append pre argv do psi.ArgumentList.Add a
               psi.UseShellExecute <- false
               // RCCL prints a version banner on stdout when a communicator starts: the
               // ranks' stdout is relayed, rank 0's contract lines only
               psi.RedirectStandardOutput <- true
               psi.Environment.["GOSSIP_RANK"] <- string r
               psi.Environment.["GOSSIP_WORLD"] <- string gpus
               psi.Environment.["GOSSIP_RDV"] <- rdv
               psi.Environment.["GOSSIP_RDV_NONCE"] <- nonce   // gp_rendezvous_id: this launch's file only
               if rehearsal then
                   psi.Environment.["NCCL_HOSTID"] <- sprintf "gossip-rehearsal-%d-%d" (Process.GetCurrentProcess().Id) r
                   psi.Environment.["NCCL_SOCKET_IFNAME"] <- "lo"
                   psi.Environment.["NCCL_IB_DISABLE"] <- "1"
               let p = new Process(StartInfo = psi)
               p.OutputDataReceived.Add(fun e ->
                   if r = 0 && not (isNull e.Data) && not (e.Data.StartsWith "RCCL version") then
                       Console.Out.WriteLine e.Data)
               p.Start() |> ignore
               p.BeginOutputReadLine()
               p |]
    let mutable failed = None
    while failed.IsNone && procs |> Array.exists (fun p -> not p.HasExited) do
        for r in 0 .. gpus - 1 do
            let p = procs.[r]
            if failed.IsNone && p.HasExited && p.ExitCode <> 0 && p.ExitCode <> 3 then failed <- Some(r, p.ExitCode)
        Threading.Thread.Sleep 200
    for r in 0 .. gpus - 1 do
        let p = procs.[r]
        if failed.IsNone && p.HasExited && p.ExitCode <> 0 && p.ExitCode <> 3 then failed <- Some(r, p.ExitCode)
    match failed with
    | Some(r, code) ->
        eprintfn "rank %d of %d failed (exit %d); stopping the other ranks" r gpus code
        for p in procs do
            if not p.HasExited then p.Kill()
    | None -> ()
    for p in procs do p.WaitForExit()
    (try IO.Directory.Delete(dir, true) with _ -> ())
    match failed with
    | Some(_, code) -> code
    | None -> procs.[0].ExitCode

let private optValue (argv: string[]) (name: string) =
    match Array.tryFindIndex ((=) name) argv with
    | Some i when i + 1 < argv.Length -> Some argv.[i + 1]
    | _ -> None

[<EntryPoint>]
let main argv =
    if argv.Length < 3 then
        eprintfn "usage: dotnet run <num_nodes> <line|full|3D|Imp3D> <gossip|push-sum> [--sync-ref|--check] [--gpus G] [--device D]"
        2
    else
        let mode = if argv.Length > 3 && (argv.[3] = "--sync-ref" || argv.[3] = "--check") then argv.[3] else ""
        let gpus =
            match optValue argv "--gpus", Environment.GetEnvironmentVariable "GOSSIP_GPUS" with
            | Some g, _ -> int g
            | None, null -> 1
            | None, g -> int g
        let device = optValue argv "--device" |> Option.map int
        let rank = match Environment.GetEnvironmentVariable "GOSSIP_RANK" with | null -> -1 | r -> int r
        if gpus > 1 && rank < 0 && mode = "" then launchRanks argv gpus device.IsSome else
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
            let lead = rank <= 0
            let rc =
                if gpus > 1 && rank >= 0 then
                    // rank process of a --gpus launch: rank 0's RCCL id through the file
                    let uid = Array.zeroCreate<byte> 128
                    let rc0 = gp_rendezvous_id (rank, Environment.GetEnvironmentVariable "GOSSIP_RDV", 600000, uid)
                    if rc0 <> 0 then rc0
                    else
                        cfg.NumGpus <- gpus
                        cfg.Device <- defaultArg device rank
                        gp_create_rank (&cfg, rank, gpus, uid, &sim)
                else
                    gp_create (&cfg, &sim)
            if rc <> 0 then
                eprintfn "[rank %d/%d] gp_create failed (%d): %s" (max rank 0) gpus rc (lastError ())
                1
            else
                if lead then printfn "%s" (starts alg)
                let mutable res = GpResult()
                let rc = gp_run (sim, &res)
                gp_destroy sim
                if rc <> 0 then
                    eprintfn "gp_run failed (%d): %s" rc (lastError ())
                    1
                elif res.Status = 0 then
                    if lead then printfn "Convergence Time: %f ms" res.ElapsedMs
                    0
                else
                    if lead then printfn "Not converged after %d rounds" res.Rounds
                    3
