"""python -m gossipprotocol_amd <num_nodes> <topology> <algorithm> [--seed S] [--max-rounds R]
                                [--gpus G] [--device D]

Same argv and stdout contract as the reference's `dotnet run` (Program.fs:32-34,
198/203, 55): prints "Gossip Starts" / "Push Sum Starts", then
"Convergence Time: %f ms".  --gpus G (or GOSSIP_GPUS=G) runs one rank process per
GPU (gossipprotocol_amd.launch; rank r on device r, or every rank on --device D
as the one-GPU rehearsal); rank 0 prints.  Same behaviour as the C++ CLI
(csrc/gossip_cli.cpp).
"""
import argparse
import os
import sys

from . import _lib as L


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    ap = argparse.ArgumentParser(prog="gossipprotocol_amd")
    ap.add_argument("num_nodes", type=int)
    ap.add_argument("topology")
    ap.add_argument("algorithm")
    ap.add_argument("--seed", type=int, default=int(os.environ.get("GOSSIP_SEED", "1")))
    ap.add_argument("--max-rounds", type=int, default=0)
    ap.add_argument("--device", type=int, default=None)
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("GOSSIP_GPUS", "1")))
    a = ap.parse_args(argv)
    if a.algorithm not in ("gossip", "push-sum"):
        print("option invalid")  # Program.fs:207
        return 2
    if a.gpus < 1:
        print("--gpus / GOSSIP_GPUS must be >= 1", file=sys.stderr)
        return 2
    # ranks started by a launcher: ours (GOSSIP_LAUNCHED) or an external one such as
    # torch.distributed.run (WORLD_SIZE / RANK in the environment) -- never launch again
    external = "WORLD_SIZE" in os.environ and not os.environ.get("GOSSIP_LAUNCHED")
    if external and int(os.environ["WORLD_SIZE"]) != a.gpus:
        seen = ", ".join(f"{k}={os.environ[k]}" for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK") if k in os.environ)
        print(f"external launcher detected ({seen}) but --gpus {a.gpus}: pass --gpus "
              f"{os.environ['WORLD_SIZE']} (or GOSSIP_GPUS) to run as its rank; refusing to run another GPU count",
              file=sys.stderr)
        return 2
    if a.gpus > 1 and not os.environ.get("GOSSIP_LAUNCHED") and not external:
        from .launch import rehearsal_env, run_ranks
        extra = (lambda r: rehearsal_env(r)) if a.device is not None else None
        return run_ranks([sys.executable, "-m", "gossipprotocol_amd"] + argv, a.gpus, env_for_rank=extra,
                         ok_codes=(0, 3))
    from .sim import Simulation
    rank = int(os.environ.get("RANK", "0")) if a.gpus > 1 else 0
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank))) if a.gpus > 1 else 0
    device = a.device if a.device is not None else local_rank
    dist = None
    if a.gpus > 1 and not os.environ.get("GOSSIP_RDV"):
        # external launcher without our rendezvous file: the RCCL id travels through a
        # gloo group on its MASTER_ADDR / MASTER_PORT (host side only)
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=a.gpus)
    try:  # the gloo group is torn down on every exit path
        try:
            sim = Simulation(a.num_nodes, a.topology, a.algorithm, seed=a.seed, max_rounds=a.max_rounds,
                             device=device, rank=rank, world=a.gpus, dist=dist,
                             rendezvous=os.environ.get("GOSSIP_RDV"))
        except L.GossipError as e:
            print(f"[rank {rank}/{a.gpus}] {e}", file=sys.stderr)
            return 2 if e.code == -1 else 1
        if rank == 0:
            print("Gossip Starts" if a.algorithm == "gossip" else "Push Sum Starts", flush=True)
        try:
            res = sim.run()
        finally:
            sim.close()
    finally:
        if dist is not None:
            dist.destroy_process_group()
    if res.status == L.GP_STATUS_CONVERGED:
        if rank == 0:
            print("Convergence Time: %f ms" % res.elapsed_ms, flush=True)
        return 0
    if rank == 0:
        print("Not converged after %d rounds (%d of %d alerts)" % (res.rounds, res.converged, res.threshold),
              flush=True)
    return 3


if __name__ == "__main__":
    sys.exit(main())
