"""Debug aid: step the LDS-resident 3D push-sum kernel (GP_KERNEL=block, experiments build) in
small batches and report, per batch, whether alerts and each state array match the oracle."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["GP_KERNEL"] = "block"
from gossipprotocol_amd import Simulation  # noqa: E402
from tests.oracle_ctypes import Oracle  # noqa: E402

n, seed = int(sys.argv[1]), int(sys.argv[2])
steps = [int(x) for x in sys.argv[3].split(",")]
sim, orc = Simulation(n, "3D", "push-sum", seed=seed, experimental=True), Oracle(n, "3D", "push-sum", seed)
print(sim.kernel_stats())
for k in steps:
    ga, oa = sim.step(k), orc.step(k)
    gs, os_ = sim.state(), orc.state()
    eq = {key: int((gs[key] != os_[key]).sum()) for key in ("s", "w", "flags")}
    print(f"after {orc.rounds}: alerts {list(ga)[:3]}.. eq={list(ga) == list(oa)} mismatches {eq} "
          f"s[:3] {gs['s'][:3]} vs {os_['s'][:3]}", flush=True)
