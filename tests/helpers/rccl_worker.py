"""One rank of a multi-process RCCL run (tests/test_gpu_rccl_multiproc.py).

    RANK=r WORLD_SIZE=W MASTER_ADDR=127.0.0.1 MASTER_PORT=p \
        python tests/helpers/rccl_worker.py OUTDIR N TOPOLOGY ALGORITHM SEED ROUNDS

Joins a gloo group (used once, to share rank 0's RCCL id -- as bench.py does under
torch.distributed.run), creates its slab with gp_create_rank on device
GP_BENCH_DEVICE (default LOCAL_RANK), steps ROUNDS rounds (every exchange is
ncclSend/ncclRecv + ncclAllReduce between the processes) and writes its alert
list and the state of its slab (above 2^24 nodes: an xxh3-128 digest of it) to
OUTDIR/rank<r>.npz.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def slab_digest(sim, first, count, chunk=1 << 24):
    """xxh3-128 over the slab's state read back in fixed chunks (c, s, w, flags per chunk)."""
    import xxhash
    h = xxhash.xxh3_128()
    for a in range(first, first + count, chunk):
        st = sim.state(a, min(chunk, first + count - a))
        for k in ("c", "s", "w", "flags"):
            h.update(st[k].tobytes())
    return h.hexdigest()


def main(argv):
    out, n, topo, alg, seed, rounds = argv[1], int(argv[2]), argv[3], argv[4], int(argv[5]), int(argv[6])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    device = int(os.environ.get("GP_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gossipprotocol_amd import Simulation
    # GP_EXP=1: the experiments build (A/B runs of its GP_* switches, scripts/)
    sim = Simulation(n, topo, alg, seed=seed, device=device, rank=rank, world=world, dist=dist,
                     experimental=os.environ.get("GP_EXP") == "1")
    alerts = sim.step(rounds)
    info = sim.info()
    if info.slab_count <= 1 << 24:
        st = sim.state(info.slab_first, info.slab_count)
    else:  # large slabs: a digest instead of the state
        st = {"digest": np.array(slab_digest(sim, info.slab_first, info.slab_count)), "count": np.int64(info.slab_count)}
    np.savez(os.path.join(out, f"rank{rank}.npz"), alerts=np.asarray(alerts, np.int64),
             first=np.int64(info.slab_first), rounds=np.int64(info.rounds),
             alerts_total=np.int64(info.alerts_total), active=np.int64(info.active), **st)
    sim.close()
    dist.barrier()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
