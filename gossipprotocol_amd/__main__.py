"""python -m gossipprotocol_amd <num_nodes> <topology> <algorithm> [--seed S] [--max-rounds R]

Same argv and stdout contract as the reference's `dotnet run` (Program.fs:32-34,
198/203, 55): prints "Gossip Starts" / "Push Sum Starts", then
"Convergence Time: %f ms".
"""
import argparse
import sys

from . import _lib as L
from .sim import Simulation


def main(argv=None):
    ap = argparse.ArgumentParser(prog="gossipprotocol_amd")
    ap.add_argument("num_nodes", type=int)
    ap.add_argument("topology")
    ap.add_argument("algorithm")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--max-rounds", type=int, default=0)
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args(argv)
    if a.algorithm not in ("gossip", "push-sum"):
        print("option invalid")  # Program.fs:207
        return 2
    try:
        sim = Simulation(a.num_nodes, a.topology, a.algorithm, seed=a.seed, max_rounds=a.max_rounds,
                         device=a.device)
    except L.GossipError as e:
        print(e, file=sys.stderr)
        return 2 if e.code == -1 else 1
    print("Gossip Starts" if a.algorithm == "gossip" else "Push Sum Starts", flush=True)
    res = sim.run()
    sim.close()
    if res.status == L.GP_STATUS_CONVERGED:
        print("Convergence Time: %f ms" % res.elapsed_ms)
        return 0
    print("Not converged after %d rounds (%d of %d alerts)" % (res.rounds, res.converged, res.threshold))
    return 3


if __name__ == "__main__":
    sys.exit(main())
