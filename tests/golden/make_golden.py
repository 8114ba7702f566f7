"""Generate tests/golden/srs_v1_golden.json from the CPU oracles.

Every case is run by the C oracle (oracle/srs_oracle.c); cases with P <= 3000
are also run by the independent pure-Python restatement (oracle/srs_py.py) and
must agree bit for bit before they are written.  The reference itself cannot
produce vectors (asynchronous F#/Akka.NET, no .NET SDK here, no tests of its
own -- SURVEY.md §4, §8c), so these fixtures pin the build's own oracle:
parity with the reference's outputs stays "parity unpinned".

    python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle.srs_py import PySim  # noqa: E402
from tests.oracle_ctypes import Oracle  # noqa: E402

# (num_nodes, topology, algorithm, seed, max_rounds)
CASES = [
    (1000, "line", "gossip", 1, 20000),      # BASELINE config 0 (C1)
    (1000, "line", "gossip", 2, 20000),
    (1000, "line", "gossip", 3, 20000),
    (60, "line", "push-sum", 1, 3000),
    (200, "full", "gossip", 1, 5000),
    (200, "full", "gossip", 2, 5000),
    (200, "full", "push-sum", 1, 5000),
    (2000, "full", "push-sum", 3, 5000),
    (1000, "3D", "gossip", 1, 20000),
    (512, "3D", "push-sum", 1, 30000),
    (1000, "Imp3D", "gossip", 1, 20000),
    (1000, "Imp3D", "gossip", 2, 20000),
    (1000, "Imp3D", "push-sum", 1, 5000),
    (1000, "Imp3D", "push-sum", 3, 5000),
    (27000, "Imp3D", "push-sum", 2, 5000),
    (1, "3D", "gossip", 1, 100),             # degenerate g = 1: no lattice edges
    (1, "Imp3D", "push-sum", 1, 100),        # g = 1: only a self random edge
    (1, "line", "gossip", 1, 100),           # P = 2
    (10**6, "3D", "push-sum", 1, 150),       # BASELINE config 1 (C2), first 150 rounds
]


def digest(alg, st):
    h = hashlib.sha256()
    if alg == "gossip":
        h.update(st["c"].astype("<i4").tobytes())
    else:
        h.update(st["s"].astype("<f8").tobytes())
        h.update(st["w"].astype("<f8").tobytes())
    h.update(st["flags"].astype("u1").tobytes())
    return h.hexdigest()


def main():
    out = []
    for n, topo, alg, seed, cap in CASES:
        o = Oracle(n, topo, alg, seed)
        alerts = o.step(cap)
        st = o.state()
        rec = {
            "num_nodes": n, "topology": topo, "algorithm": alg, "seed": seed, "max_rounds": cap,
            "population": o.P, "threshold": o.T, "seed_node": o.seed_node,
            "rounds": len(alerts), "alerts_total": int(sum(alerts)),
            "converged": bool(sum(alerts) >= o.T),
            "alerts_per_round": [int(a) for a in alerts],
            "state_sha256": digest(alg, st),
            "head": {k: st[k][:16].tolist() for k in ("c", "s", "w", "flags")},
            "python_crosscheck": False,
        }
        if o.P <= 3000:
            p = PySim(n, topo, alg, seed)
            pa = p.step(cap)
            assert pa == rec["alerts_per_round"], (n, topo, alg, seed)
            if alg == "gossip":
                assert list(st["c"]) == p.c
            else:
                assert list(st["s"]) == p.s and list(st["w"]) == p.w
            assert list(st["flags"]) == p.flags()
            rec["python_crosscheck"] = True
        # sparse per-round alerts are long for slow cases: keep them all (ints)
        out.append(rec)
        print(n, topo, alg, seed, "P", o.P, "rounds", rec["rounds"], "conv", rec["converged"],
              "xcheck", rec["python_crosscheck"], flush=True)
        o.close()
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "srs_v1_golden.json")
    with open(path, "w") as f:
        json.dump({"spec": "SRS v1 (SURVEY.md Appendix B)", "generator": "tests/golden/make_golden.py",
                   "cases": out}, f, separators=(",", ":"))
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
