"""Generate tests/golden/runs_1e8.json: whole runs to convergence at BASELINE.json's
1e8 sizes, from the C oracle (oracle/srs_oracle.c, OpenMP).

    python tests/golden/make_golden_runs.py [case ...]     # cases: c2 c4 c5_1e8 (default: all)

Per case: the per-round alert counts of the whole run (the scheduler's Alert
stream, Program.fs:51-56, under SRS v1), the convergence round, and an xxh3-128
digest of the final state (s, w, flags in 2^24-node chunks, the same digest
tests/helpers/rccl_worker.py slab_digest computes from the product).  The GPU
tests run the product to convergence and compare all three -- the whole-network
oracle comparison at these sizes without re-running the oracle (minutes of CPU
per run) inside the GPU suite.  Fixtures of the build's own oracle: the
reference produces no vectors, so parity with it stays
"parity unpinned".

C2: push-sum, 3D lattice, n = 1e6 (g = 100, P = 1,000,000), seed 1.
C4: push-sum, full topology, n = 1e8 (P = 100,000,001), seed 1.
C5@1e8: push-sum, Imp3D, n = 1e8 (g = 465, P = 100,544,625), seed 1.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from tests.oracle_ctypes import Oracle  # noqa: E402

CASES = {"c2": (10**6, "3D", "push-sum", 1), "c4": (10**8, "full", "push-sum", 1), "c5_1e8": (10**8, "Imp3D", "push-sum", 1)}
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "runs_1e8.json")


def digest(read, P, chunk=1 << 24):
    import xxhash
    h = xxhash.xxh3_128()
    for a in range(0, P, chunk):
        st = read(a, min(chunk, P - a))
        for k in ("c", "s", "w", "flags"):
            h.update(np.ascontiguousarray(st[k]).tobytes())
    return h.hexdigest()


def main(names):
    out = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for name in names:
        n, topo, alg, seed = CASES[name]
        t0 = time.time()
        orc = Oracle(n, topo, alg, seed, threads=int(os.environ.get("OMP_NUM_THREADS", "0") or 0))
        alerts = []
        while orc.alerts_total < orc.T:
            a = orc.step(64)
            if not a:
                break
            alerts += a
            print(f"[{name}] round {orc.rounds}: alerts {orc.alerts_total} of {orc.T} ({time.time() - t0:.0f} s)",
                  file=sys.stderr, flush=True)
        out[name] = {"num_nodes": n, "topology": topo, "algorithm": alg, "seed": seed, "population": orc.P,
                     "threshold": orc.T, "rounds": orc.rounds, "alerts_total": orc.alerts_total,
                     "alerts_per_round": alerts, "final_state_xxh3_128": digest(orc.state, orc.P),
                     "oracle_seconds": round(time.time() - t0, 1)}
        orc.close()
        with open(OUT, "w") as f:
            json.dump(out, f)
        print(f"[{name}] converged in {out[name]['rounds']} rounds", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main(sys.argv[1:] or list(CASES))
