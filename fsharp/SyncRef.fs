/// SyncRef: the synchronous-round mode of the reference (SRS v1, SURVEY.md
/// Appendix B) restated in F#, with the same Philox4x32-10 stream as the HIP
/// kernels and the C oracle, so that `dotnet run -- --sync-ref ...` can check
/// libgossip_hip bit for bit on a host with a .NET SDK.
/// UNVERIFIED here (no .NET SDK in the image); the operative oracle is
/// oracle/srs_oracle.c, cross-checked by oracle/srs_py.py.
module SyncRef

let private philox (c0: uint32, c1: uint32, c2: uint32, c3: uint32) (k0: uint32, k1: uint32) =
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

/// U(m) = floor(((y<<32)|x) * m / 2^64); ctr = (node, round, stream, 0), key = seed.
let uniform (seed: uint64) (stream: uint32) (node: uint32) (round: uint32) (m: uint32) =
    let x, y = philox (node, round, stream, 0u) (uint32 seed, uint32 (seed >>> 32))
    let lo = uint64 x * uint64 m
    let hi = uint64 y * uint64 m + (lo >>> 32)
    uint32 (hi >>> 32)

/// Lattice slot order of the reference: x-1, x+1, y+1, y-1, z+1, z-1.
let latticeNeighbours (g: int) (id: int) =
    let g2 = g * g
    let x, y, z = id / g2, (id / g) % g, id % g
    [| if x > 0 then yield id - g2
       if x < g - 1 then yield id + g2
       if y < g - 1 then yield id + g
       if y > 0 then yield id - g
       if z < g - 1 then yield id + 1
       if z > 0 then yield id - 1 |]

/// One synchronous gossip round on the 3D / Imp3D lattice (SRS v1 B.3);
/// `nbrs` is the slot-ordered neighbour array, `live` the injector list.
let gossipRound (seed: uint64) (r: uint32) (seedNode: int) (nbrs: int[][]) (c: int[]) (live: ResizeArray<int>) =
    let conv = c |> Array.map (fun v -> v >= 11)
    let inc = Array.zeroCreate c.Length
    for i in 0 .. c.Length - 1 do
        if (i = seedNode || c.[i] >= 1) && c.[i] <= 10 && nbrs.[i].Length > 0 then
            let t = nbrs.[i].[int (uniform seed 2u (uint32 i) r (uint32 nbrs.[i].Length))]
            if not conv.[t] then inc.[t] <- inc.[t] + 1
    if live.Count > 0 then
        let t = live.[int (uniform seed 4u 0u r (uint32 live.Count))]
        if conv.[t] then live.Remove t |> ignore else inc.[t] <- inc.[t] + 1
    let mutable alerts = 0
    for j in 0 .. c.Length - 1 do
        if inc.[j] > 0 then
            if c.[j] <= 10 && c.[j] + inc.[j] > 10 then alerts <- alerts + 1
            c.[j] <- c.[j] + inc.[j]
    alerts
