"""Full push-sum parity of the experiments build under the current GP_* overrides (e.g. GP_FB_FUSED=0):
small populations against the C oracle through convergence, and P = 1e8 against the product
library (itself oracle-checked at that size, tests/test_gpu_baseline_sizes.py) state for state."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gossipprotocol_amd import Simulation  # noqa: E402
from tests.oracle_ctypes import Oracle  # noqa: E402

for n in (4095, 4097, 65537, 1000000):
    sim, orc = Simulation(n, "full", "push-sum", seed=3, experimental=True), Oracle(n, "full", "push-sum", 3)
    assert sim.step(5000) == orc.step(5000), n
    a, b = sim.state(), orc.state()
    for k in ("s", "w", "flags"):
        assert np.array_equal(a[k], b[k]), (n, k)
    sim.close()
    orc.close()
    print("oracle ok", n, flush=True)
n = 10**8
with Simulation(n, "full", "push-sum", seed=1, experimental=True) as v, Simulation(n, "full", "push-sum", seed=1) as p:
    for _ in range(4):
        assert v.step(10) == p.step(10)
        for lo in range(0, n, 1 << 25):
            a, b = v.state(lo, min(1 << 25, n - lo)), p.state(lo, min(1 << 25, n - lo))
            for k in ("s", "w", "flags"):
                assert np.array_equal(a[k], b[k]), (lo, k)
    print("1e8 vs product ok (40 rounds)", flush=True)
