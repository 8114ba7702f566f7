"""Bit-exact check of an experiments-build library variant against the C oracle
(experiment tool, run on the GPU box; the variant is GOSSIP_HIP_LIB_EXPERIMENT).

    python tools/variant_parity.py <n> <topology> <algorithm> <rounds> [seed]
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
    ga, oa = sim.step(rounds), orc.step(rounds)
    assert ga == oa, "per-round alerts differ from the oracle"
    gs, os_ = sim.state(), orc.state()
    for k in ("c", "s", "w", "flags"):
        assert np.array_equal(gs[k], os_[k]), f"state '{k}' differs from the oracle"
    print(f"variant parity ok: {os.environ.get('GOSSIP_HIP_LIB_EXPERIMENT')} {topo} {alg} n={n} rounds={len(ga)}")


if __name__ == "__main__":
    main()
