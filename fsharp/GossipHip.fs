/// P/Invoke binding of libgossip_hip.so (include/gossip_hip.h).
/// Blittable structs only, Cdecl, no marshalling code needed.
/// UNVERIFIED in this repository's CI: no .NET SDK exists in the build image.
module GossipHip

open System
open System.Runtime.InteropServices

[<Literal>]
let Lib = "gossip_hip"

[<Struct; StructLayout(LayoutKind.Sequential)>]
type GpConfig =
    val mutable NumNodes: int64
    val mutable Topology: int32
    val mutable Algorithm: int32
    val mutable Seed: uint64
    val mutable NumGpus: int32
    val mutable Device: int32
    val mutable MaxRounds: int64
    val mutable Flags: int32
    val mutable Reserved: int32

[<Struct; StructLayout(LayoutKind.Sequential)>]
type GpResult =
    val mutable Rounds: int64
    val mutable Converged: int64
    val mutable Population: int64
    val mutable Threshold: int64
    val mutable ElapsedMs: double
    val mutable NodeUpdatesPerS: double
    val mutable HbmBytesAlg: double
    val mutable Status: int32
    val mutable Reserved: int32

[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern int gp_parse_topology(string s)

[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern int gp_parse_algorithm(string s)

[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern int gp_create(GpConfig& cfg, nativeint& sim)

/// Multi-GPU, one process per GPU: rank 0 publishes its RCCL id at `path`, the
/// other ranks read it (include/gossip_hip.h gp_rendezvous_id); then every rank
/// joins with gp_create_rank.
[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern int gp_rendezvous_id(int rank, string path, int timeoutMs, byte[] uniqueId)

[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern int gp_create_rank(GpConfig& cfg, int rank, int world, byte[] uniqueId, nativeint& sim)

[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern int gp_run(nativeint sim, GpResult& result)

[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern int64 gp_step(nativeint sim, int64 nrounds, int64[] alertsPerRound)

[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern int gp_read_state(nativeint sim, int64 first, int64 count, int32[] c, double[] s, double[] w, byte[] flags)

[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern void gp_destroy(nativeint sim)

[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern nativeint gp_last_error()

let lastError () = Marshal.PtrToStringAnsi(gp_last_error ())
