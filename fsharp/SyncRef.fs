/// SyncRef: the synchronous-round mode of the reference -- SRS v1 (SURVEY.md
/// Appendix B) restated in F# next to the reference's own language, with the
/// same Philox4x32-10 stream as the HIP kernels (gossipprotocol_amd/csrc) and
/// the C oracle (oracle/srs_oracle.c).  `dotnet run -- <n> <topology>
/// <algorithm> --sync-ref` runs it alone; `--check` runs it in lock step with
/// libgossip_hip.so and compares per-round alerts and the final state bit for
/// bit (Program.fs in this directory).
///
/// Every block cites the lines of /root/reference/Project2/Program.fs (quoted
/// as Program.fs:N) it restates.  Written for clarity at small N (lists per
/// receiver, an O(P) injector list), not speed.
///
/// UNVERIFIED here: no .NET SDK exists in the build image or on the GPU boxes.
/// It was reviewed line by line against oracle/srs_oracle.c (same population
/// rules, slot orders, streams, fold order and ratio test); the operative
/// oracle is the C one, cross-checked by oracle/srs_py.py.
module SyncRef

open System
open System.Collections.Generic

// ---------------------------------------------------------------- RNG (SRS v1 B.2)
/// Random123 Philox4x32 with 10 rounds; returns output words 0 and 1.
/// Replaces `new Random()` (Program.fs:86,103,128,130,152,193,221,259,263).
let philox (c0: uint32, c1: uint32, c2: uint32, c3: uint32) (k0: uint32, k1: uint32) =
    let mutable a = c0
    let mutable b = c1
    let mutable c = c2
    let mutable d = c3
    let mutable x = k0
    let mutable y = k1
    for r in 0 .. 9 do
        if r > 0 then
            x <- x + 0x9E3779B9u
            y <- y + 0xBB67AE85u
        let p0 = uint64 0xD2511F53u * uint64 a
        let p1 = uint64 0xCD9E8D57u * uint64 c
        let na = uint32 (p1 >>> 32) ^^^ b ^^^ x
        let nc = uint32 (p0 >>> 32) ^^^ d ^^^ y
        b <- uint32 p1
        d <- uint32 p0
        a <- na
        c <- nc
    a, b

/// Streams (Philox counter word 2).
let STOPO, SSTART, SGOSSIP, SPUSHSUM, SINJECT = 0u, 1u, 2u, 3u, 4u

/// U(m) = floor(((y<<32)|x) * m / 2^64) with ctr = (node, round, stream, 0), key = seed.
let uniform (seed: uint64) (stream: uint32) (node: uint32) (round: uint32) (m: uint32) =
    let x, y = philox (node, round, stream, 0u) (uint32 seed, uint32 (seed >>> 32))
    let lo = uint64 x * uint64 m
    let hi = uint64 y * uint64 m + (lo >>> 32)
    uint32 (hi >>> 32)

// ---------------------------------------------------------------- population (SRS v1 B.1)
type Topology =
    | Line = 0
    | Full = 1
    | Grid3D = 2
    | Imp3D = 3

type Algorithm =
    | Gossip = 0
    | PushSum = 1

/// Case-sensitive like Program.fs:180,209,238,258 ("imp3D" accepted as BASELINE's alias).
let parseTopology (s: string) =
    match s with
    | "line" -> Some Topology.Line
    | "full" -> Some Topology.Full
    | "3D" -> Some Topology.Grid3D
    | "Imp3D" | "imp3D" -> Some Topology.Imp3D
    | _ -> None

/// Program.fs:196,202 ("push-sum", not "push sum").
let parseAlgorithm (s: string) =
    match s with
    | "gossip" -> Some Algorithm.Gossip
    | "push-sum" -> Some Algorithm.PushSum
    | _ -> None

/// Exact ceil(cbrt n): Program.fs:239-240 uses Math.Cbrt + ceil, which is libm
/// dependent (Q3); SRS v1 pins it with integer arithmetic.
let icbrtCeil (n: int64) =
    let mutable g = int64 (Math.Cbrt(float n))
    while g > 0L && g * g * g >= n do
        g <- g - 1L
    while g * g * g < n do
        g <- g + 1L
    g

/// (P, T, g): line / full spawn nodes+1 actors and stop at `nodes` alerts
/// (Program.fs:170-171,53); 3D / Imp3D P = T = g^3 (Program.fs:239; SRS D1).
let resolve (n: int64) (topo: Topology) =
    match topo with
    | Topology.Line
    | Topology.Full -> n + 1L, n, 0L
    | _ ->
        let g = icbrtCeil n
        g * g * g, g * g * g, g

// ---------------------------------------------------------------- topology
type Net =
    { Topo: Topology
      P: int
      T: int
      G: int
      Seed: uint64
      /// Imp3D random neighbour per node: Random().Next(0, nodes-1) -> [0, P-2]
      /// (Program.fs:258-260), drawn once from the TOPO stream.
      Rnd: int[] }

let makeNet (n: int64) (topo: Topology) (seed: uint64) =
    let P, T, g = resolve n topo
    let P, T, g = int P, int T, int g
    let rnd =
        if topo = Topology.Imp3D then
            Array.init P (fun i -> int (uniform seed STOPO (uint32 i) 0u (uint32 (P - 1))))
        else
            [||]
    { Topo = topo; P = P; T = T; G = g; Seed = seed; Rnd = rnd }

/// Lattice slot order of the reference: x-1, x+1, y+1, y-1, z+1, z-1, each only
/// if in range (Program.fs:246-257), id = x*g^2 + y*g + z.
let latticeNeighbours (g: int) (id: int) =
    let g2 = g * g
    let x, y, z = id / g2, (id / g) % g, id % g
    [| if x > 0 then yield id - g2
       if x < g - 1 then yield id + g2
       if y < g - 1 then yield id + g
       if y > 0 then yield id - g
       if z < g - 1 then yield id + 1
       if z > 0 then yield id - 1 |]

/// Line: node 0 -> [1], the last node -> [P-2], else [i-1; i+1] (Program.fs:182-191).
let lineNeighbours (P: int) (i: int) =
    if P = 1 then [||]
    elif i = 0 then [| 1 |]
    elif i = P - 1 then [| P - 2 |]
    else [| i - 1; i + 1 |]

let degree (net: Net) (i: int) =
    match net.Topo with
    | Topology.Line -> (lineNeighbours net.P i).Length
    | Topology.Full -> net.P - 1 // Program.fs:211-216: every j <> i
    | Topology.Grid3D -> (latticeNeighbours net.G i).Length
    | _ -> (latticeNeighbours net.G i).Length + 1

/// Slot k of node i -> (target, isRandom).  Full: the k-th of the ascending
/// j <> i (Program.fs:213-215); Imp3D: the slot after the lattice ones is the
/// random edge (Program.fs:258-260).
let slotTarget (net: Net) (i: int) (k: int) =
    match net.Topo with
    | Topology.Line -> (lineNeighbours net.P i).[k], false
    | Topology.Full -> (if k < i then k else k + 1), true
    | Topology.Grid3D -> (latticeNeighbours net.G i).[k], false
    | _ ->
        let nb = latticeNeighbours net.G i
        if k = nb.Length then net.Rnd.[i], true else nb.[k], false

/// Position of `sender` in the target's own lattice / line slot list: the
/// canonical order in which the target folds lattice messages.
let latticeKey (net: Net) (target: int) (sender: int) =
    let nb =
        if net.Topo = Topology.Line then lineNeighbours net.P target else latticeNeighbours net.G target
    uint64 (Array.findIndex ((=) sender) nb)

// ---------------------------------------------------------------- state
type Sim =
    { Net: Net
      Alg: Algorithm
      SeedNode: int
      mutable Round: uint32
      mutable AlertsTotal: int64
      mutable Done: bool
      // gossip: rumour counters (Program.fs:68), injector list (Program.fs:147-148)
      C: int[]
      Live: List<int>
      // push-sum: sum = id, weight = 1, count = 1 (Program.fs:67,71,78,174)
      S: float[]
      W: float[]
      Active: bool[]
      Conv: bool[]
      Cnt: int[] }

let create (n: int64) (topo: Topology) (alg: Algorithm) (seed: uint64) =
    let net = makeNet n topo seed
    let P = net.P
    // choice = Random().Next(0, nodes) (Program.fs:193,221,263)
    let seedNode = int (uniform seed SSTART 0u 0u (uint32 net.T))
    let gossip = alg = Algorithm.Gossip
    let injector = gossip && topo <> Topology.Full // Program.fs:200,271 (not 224-228)
    let sim =
        { Net = net
          Alg = alg
          SeedNode = seedNode
          Round = 0u
          AlertsTotal = 0L
          Done = false
          C = Array.zeroCreate (if gossip then P else 0)
          Live = (if injector then List<int>(seq { 0 .. net.T - 1 }) else List<int>())
          S = (if gossip then [||] else Array.init P float)
          W = (if gossip then [||] else Array.create P 1.0)
          Active = Array.init (if gossip then 0 else P) (fun i -> i = seedNode)
          Conv = Array.zeroCreate (if gossip then 0 else P)
          Cnt = Array.create (if gossip then 0 else P) 1 }
    sim

// ---------------------------------------------------------------- gossip (SRS v1 B.3)
/// Process1 (Program.fs:84-89): a node that has the rumour and has heard it at
/// most 10 times (or the seed) picks a uniform neighbour and sends unless the
/// target is converged in the round-start snapshot (`dictionary`, Program.fs:87).
/// Injector (Program.fs:141-163): k-th id of the live list; remove if converged,
/// else deliver.  Process2 (Program.fs:91-98): the receipt that finds
/// rumours = 10 alerts.
let private gossipRound (sim: Sim) =
    let net = sim.Net
    let r = sim.Round
    let c = sim.C
    let conv = c |> Array.map (fun v -> v >= 11)
    let inc = Array.zeroCreate net.P
    for i in 0 .. net.P - 1 do
        let ci = c.[i]
        if (i = sim.SeedNode || ci >= 1) && ci <= 10 then
            let deg = degree net i
            if deg > 0 then
                let k = int (uniform net.Seed SGOSSIP (uint32 i) r (uint32 deg))
                let t, _ = slotTarget net i k
                if not conv.[t] then inc.[t] <- inc.[t] + 1
    if sim.Live.Count > 0 then
        let k = int (uniform net.Seed SINJECT 0u r (uint32 sim.Live.Count))
        let t = sim.Live.[k] // the list stays ascending: the k-th live id
        if conv.[t] then sim.Live.RemoveAt k else inc.[t] <- inc.[t] + 1
    let mutable alerts = 0L
    for j in 0 .. net.P - 1 do
        if inc.[j] > 0 then
            if c.[j] <= 10 && c.[j] + inc.[j] > 10 then alerts <- alerts + 1L
            c.[j] <- c.[j] + inc.[j]
    alerts

// ---------------------------------------------------------------- push-sum (SRS v1 B.4)
/// MainPushSum (Program.fs:101-131): every active node halves (sum, weight) and
/// sends the halves to one uniform neighbour (Program.fs:104-106,125-128); each
/// receiver adds its messages in canonical order -- own half, lattice messages
/// in its own slot order, then random-edge / full messages by ascending sender
/// id -- and runs the ratio test against the round-start ratio with 1e-10
/// (Program.fs:114-123; SRS D5 fixes Q11), count 3 converges and alerts
/// (Program.fs:121-123).  Converged nodes keep sending (D6).
let private pushSumRound (sim: Sim) =
    let net = sim.Net
    let r = sim.Round
    let P = net.P
    let inbox = Array.init P (fun _ -> List<struct (uint64 * int)>())
    let sMsg = Array.zeroCreate P
    let wMsg = Array.zeroCreate P
    for i in 0 .. P - 1 do
        if sim.Active.[i] then
            let deg = degree net i
            if deg > 0 then
                let k = int (uniform net.Seed SPUSHSUM (uint32 i) r (uint32 deg))
                let t, isRandom = slotTarget net i k
                let key = if isRandom then (1UL <<< 40) + uint64 i else latticeKey net t i
                inbox.[t].Add(struct (key, i))
                sMsg.[i] <- sim.S.[i] * 0.5
                wMsg.[i] <- sim.W.[i] * 0.5
    let mutable alerts = 0L
    for j in 0 .. P - 1 do
        let s0, w0 = sim.S.[j], sim.W.[j]
        let halve = sim.Active.[j] && degree net j > 0
        let mutable accS = if halve then s0 * 0.5 else s0
        let mutable accW = if halve then w0 * 0.5 else w0
        let msgs = inbox.[j]
        if msgs.Count > 0 then
            msgs.Sort(fun (struct (a, _)) (struct (b, _)) -> compare a b)
            for struct (_, i) in msgs do
                accS <- accS + sMsg.[i]
                accW <- accW + wMsg.[i]
            let rOld = s0 / w0
            let rNew = accS / accW
            if not sim.Conv.[j] then
                let cnt = if abs (rNew - rOld) > 1e-10 then 0 else sim.Cnt.[j] + 1
                if cnt = 3 then
                    sim.Conv.[j] <- true
                    alerts <- alerts + 1L
                sim.Cnt.[j] <- cnt
            sim.Active.[j] <- true
        sim.S.[j] <- accS
        sim.W.[j] <- accW
    alerts

// ---------------------------------------------------------------- driver
/// Scheduler (Program.fs:41-61): count alerts, stop after the round in which
/// they reach T.  Runs at most `nrounds` rounds; returns the per-round alerts.
let step (sim: Sim) (nrounds: int) =
    let out = List<int64>()
    while out.Count < nrounds && not sim.Done do
        let a = if sim.Alg = Algorithm.Gossip then gossipRound sim else pushSumRound sim
        out.Add a
        sim.AlertsTotal <- sim.AlertsTotal + a
        sim.Round <- sim.Round + 1u
        if sim.AlertsTotal >= int64 sim.Net.T then sim.Done <- true
    out.ToArray()

/// Node state in the C-ABI's readback format (gp_read_state): c, s, w, flags
/// (bit0 active, bit1 converged, bits2-3 push-sum count).
let state (sim: Sim) =
    let P = sim.Net.P
    if sim.Alg = Algorithm.Gossip then
        let flags =
            Array.init P (fun i ->
                let ci = sim.C.[i]
                let act = (i = sim.SeedNode || ci >= 1) && ci <= 10
                byte ((if act then 1 else 0) ||| (if ci >= 11 then 2 else 0)))
        Array.copy sim.C, Array.zeroCreate<float> P, Array.zeroCreate<float> P, flags
    else
        let flags =
            Array.init P (fun i ->
                byte ((if sim.Active.[i] then 1 else 0) ||| (if sim.Conv.[i] then 2 else 0) ||| (sim.Cnt.[i] <<< 2)))
        Array.zeroCreate<int> P, Array.copy sim.S, Array.copy sim.W, flags
