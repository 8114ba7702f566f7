"""Run one configuration to convergence on the HIP path and record the run
(experiment tool): rounds, wall time, per-round alerts, per-round kernel time.

    python tools/converge.py [n] [topology] [algorithm] [seed] [out.json]

The round loop is the library's own (gp_step batches of 1024 rounds, one host
synchronisation per batch); kernel times come from HIP events around every
round kernel.  The result JSON carries the convergence round (SRS v1: the round
in which the cumulative alerts reach T, Program.fs:53), the wall time from the
first round to convergence (the reference's Stopwatch, Program.fs:194,54), the
activation round (every node active) and the alert curve.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gossipprotocol_amd import Simulation  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10**9
    topo = sys.argv[2] if len(sys.argv) > 2 else "Imp3D"
    alg = sys.argv[3] if len(sys.argv) > 3 else "push-sum"
    seed = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    out = sys.argv[5] if len(sys.argv) > 5 else None
    t = time.perf_counter()
    sim = Simulation(n, topo, alg, seed=seed, kernel_timing=True)
    t_create = time.perf_counter() - t
    P, T = sim.population, sim.threshold
    alerts, kms, active_round = [], [], None
    t0 = time.perf_counter()
    while True:
        # 8-round steps until every node is active, so the activation round is exact to 8
        # (bench.py's pre-roll does the same); then 1024-round batches
        a = sim.step(8 if active_round is None and alg == "push-sum" else 1024)
        ms, k, name = sim.kernel_stats(reset=True)
        alerts += a
        kms.append((len(a), ms))
        if active_round is None and alg == "push-sum" and sim.info().active >= P:
            active_round = sim.rounds
        if not a or sim.alerts_total >= T:
            break
        if len(a) == 8 and active_round is None:
            continue
        print(f"[converge] round {sim.rounds}: alerts {sim.alerts_total} of {T} "
              f"({time.perf_counter() - t0:.1f} s)", file=sys.stderr, flush=True)
    wall = time.perf_counter() - t0
    rec = {"num_nodes": n, "topology": topo, "algorithm": alg, "seed": seed, "population": P, "threshold": T,
           "rounds": sim.rounds, "converged": sim.alerts_total >= T, "wall_s": wall, "create_s": t_create,
           "kernel": name, "kernel_ms_total": sum(m for _, m in kms),
           "activation_round": active_round,
           "node_updates_per_s": P * sim.rounds / wall,
           "alerts_per_round": alerts}
    sim.close()
    s = json.dumps(rec)
    if out:
        with open(out, "w") as f:
            f.write(s)
    summary = {k: v for k, v in rec.items() if k != "alerts_per_round"}
    print(json.dumps(summary), flush=True)


if __name__ == "__main__":
    main()
