import os, sys
sys.path.insert(0, os.getcwd())
os.environ["GP_KERNEL"] = sys.argv[1] if len(sys.argv) > 1 else "col"
os.environ["GP_XSEGS"] = sys.argv[2] if len(sys.argv) > 2 else "2"
from gossipprotocol_amd import Simulation
from tests.oracle_ctypes import Oracle
import numpy as np
orc = Oracle(125000, "Imp3D", "gossip", 7)
oa = orc.step(300)
oc = orc.state()["c"]
for rep in range(4):
    sim = Simulation(125000, "Imp3D", "gossip", seed=7)
    ga = []
    first_bad_state = None
    for r in range(30):
        ga += sim.step(1)
    st = sim.state()
    o2 = Oracle(125000, "Imp3D", "gossip", 7); o2.step(30); oc30 = o2.state()["c"]; o2.close()
    bad = np.nonzero(st["c"] != oc30)[0]
    d = [i for i in range(len(ga)) if ga[i] != oa[i]]
    print(f"rep {rep}: alert diffs at rounds {d[:5]}; c mismatches after 30 rounds: {len(bad)} first {bad[:5]} gpu {st['c'][bad[:5]]} orc {oc30[bad[:5]]}", flush=True)
    sim.close()
