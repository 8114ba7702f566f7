"""Steady-state round-kernel timing probe (experiment tool).

    python tools/perf_round.py [n] [topology] [algorithm] [rounds]

Advances the simulation until every node is active (push-sum) or for a fixed
number of rounds (gossip), then times `rounds` rounds with HIP events around
the round kernel.  Prints ms/round and algorithmic GB/s.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gossipprotocol_amd import Simulation  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10**9
    topo = sys.argv[2] if len(sys.argv) > 2 else "Imp3D"
    alg = sys.argv[3] if len(sys.argv) > 3 else "push-sum"
    k = int(sys.argv[4]) if len(sys.argv) > 4 else 10
    t = time.perf_counter()
    # the experiments build (GP_* overrides, ablation builds) when asked for
    exp = bool(os.environ.get("GOSSIP_HIP_LIB_EXPERIMENT") or os.environ.get("GP_EXP"))
    s = Simulation(n, topo, alg, kernel_timing=True, experimental=exp)
    tc = time.perf_counter() - t
    P = s.population
    s.kernel_stats(reset=True)
    pre = 0
    t = time.perf_counter()
    if alg == "push-sum":
        while s.info().active < P and pre < 3000:
            pre += len(s.step(8))
    else:
        pre += len(s.step(40))
    s.sync()
    tp = time.perf_counter() - t
    pms, pk, _ = s.kernel_stats(reset=True)
    t = time.perf_counter()
    got = s.step(k)
    s.sync()
    wall = time.perf_counter() - t
    ms, kk, name = s.kernel_stats()
    bpn = s.alg_bytes_per_node()
    print(f"{topo} {alg} P={P} create {tc:.2f}s preroll {pre} rounds {tp:.2f}s ({pms / max(pk, 1):.2f} ms/kernel) | "
          f"{name}: {ms / kk:.3f} ms/round kernel, wall {wall * 1e3 / len(got):.3f} ms/round, "
          f"{P * len(got) / wall:.3e} node-updates/s, alg {bpn * P / (ms / kk * 1e-3) / 1e9:.0f} GB/s", flush=True)
    s.close()
    if P <= 2 * 10**7 and os.environ.get("GP_NOEV", "1") != "0":
        # small populations: wall per round without per-round HIP events (their
        # recording is itself a visible share of a tens-of-microseconds round)
        s = Simulation(n, topo, alg, experimental=exp)
        pre2 = 0
        while pre2 < pre:
            pre2 += len(s.step(min(8, pre - pre2)))
        s.sync()
        t = time.perf_counter()
        got = s.step(k)
        s.sync()
        wall = time.perf_counter() - t
        print(f"  no events: wall {wall * 1e3 / len(got):.4f} ms/round over {len(got)} rounds", flush=True)
        s.close()


if __name__ == "__main__":
    main()
