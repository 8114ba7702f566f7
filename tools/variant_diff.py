"""First round where an experiments-build variant (GOSSIP_HIP_LIB_EXPERIMENT) departs
from the C oracle, and the differing nodes (experiment / debugging tool).

    python tools/variant_diff.py <n> <topology> <algorithm> <max_rounds> [seed]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gossipprotocol_amd import Simulation  # noqa: E402
from tests.oracle_ctypes import Oracle  # noqa: E402


def main():
    n, topo, alg, rounds = int(sys.argv[1]), sys.argv[2], sys.argv[3], int(sys.argv[4])
    seed = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    sim = Simulation(n, topo, alg, seed=seed, experimental=True)
    orc = Oracle(n, topo, alg, seed)
    g = sim.info().grid
    for r in range(rounds):
        ga, oa = sim.step(1), orc.step(1)
        gs, os_ = sim.state(), orc.state()
        bad = np.zeros(len(gs["s"]), bool)
        for k in ("c", "s", "w", "flags"):
            bad |= gs[k] != os_[k]
        if bad.any() or ga != oa:
            ids = np.nonzero(bad)[0]
            print(f"round {r}: alerts gpu {ga} oracle {oa}; {len(ids)} nodes differ")
            for i in ids[:12]:
                xyz = (i // (g * g), (i // g) % g, i % g) if g else ()
                print(f"  node {i} xyz {xyz} tile {i // 1024} off {i % 1024} | gpu s {gs['s'][i]!r} w {gs['w'][i]!r} "
                      f"f {gs['flags'][i]} | oracle s {os_['s'][i]!r} w {os_['w'][i]!r} f {os_['flags'][i]}")
            return
    print("no difference in", rounds, "rounds")


if __name__ == "__main__":
    main()
