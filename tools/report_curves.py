"""Report-curve harness: convergence of every topology x
algorithm pair at the node counts of the reference's Report.pdf plots, over many
seeds, on the product path (libgossip_hip.so through gossipprotocol_amd).

    python tools/report_curves.py [--seeds S] [--nodes 100,200,...] [--out DIR]

The reference reports only wall-clock convergence times of its asynchronous Akka
run on an unknown Mac (Report.pdf p.1 gossip, p.2 push-sum; digitised in SURVEY.md
§6), so no number is comparable.  What is comparable is the qualitative ordering
the report and README.md:3 state: full converges fastest, line slowest, Imp3D no
slower than 3D.  This tool measures convergence rounds (the synchronous
equivalent of the reference's `Convergence Time`, Program.fs:53-55) and the GPU
wall time, and checks those orderings per node count on the seed medians.

`sweep` takes the simulator as a callable, so tests can drive it with the CPU
oracle at small sizes; the command line uses the product only.
"""
import argparse
import json
import os
import statistics
import sys
import time

TOPOLOGIES = ("line", "full", "3D", "Imp3D")
ALGORITHMS = ("gossip", "push-sum")
REPORT_NODES = tuple(range(100, 1001, 100))

# Digitised Report.pdf values (ms); None = occluded / absent marker.
REPORT_MS = {
    "gossip": {
        "line": [362, 394, 756, 1110, 1594, 1923, 2357, 3080, 3706, None],
        "full": [175, 152, 180, 187, 212, 212, 212, 217, 249, 252],
        "3D": [340, 554, 561, 441, 511, 935, 1005, 1706, 1870, 1120],
        "Imp3D": [499, 322, 377, 541, 505, 843, 761, 1419, 1160, 1192],
    },
    "push-sum": {
        "line": [215, 270, 2390, 2463, 6930, 1945, 1925, 3980, 5467, 8340],
        "full": [None] * 10,
        "3D": [None] * 6 + [300, 1189, 330, 1110],
        "Imp3D": [175, 175, 192, 209, 203, 220, 316, 990, 321, 280],
    },
}


def product_runner(device=0, max_rounds=10**6):
    """Runner over the HIP path: (n, topology, algorithm, seed) -> (rounds, converged, ms)."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from gossipprotocol_amd import Simulation
    from gossipprotocol_amd import _lib as L

    def run(n, topology, algorithm, seed):
        with Simulation(n, topology, algorithm, seed=seed, max_rounds=max_rounds, device=device) as s:
            r = s.run()
            return int(r.rounds), r.status == L.GP_STATUS_CONVERGED, float(r.elapsed_ms)
    return run


def sweep(runner, nodes=REPORT_NODES, seeds=(1, 2, 3, 4, 5), topologies=TOPOLOGIES,
          algorithms=ALGORITHMS, progress=None):
    """Runs every (algorithm, topology, n, seed); returns
    {alg: {topo: [{"n", "rounds": [...], "ms": [...], "converged": k, "median_rounds"}]}}."""
    table = {}
    for alg in algorithms:
        table[alg] = {}
        for topo in topologies:
            rows = []
            for n in nodes:
                rounds, ms, conv = [], [], 0
                for sd in seeds:
                    r, ok, t = runner(n, topo, alg, sd)
                    rounds.append(r)
                    ms.append(t)
                    conv += int(ok)
                rows.append({"n": n, "rounds": rounds, "ms": ms, "converged": conv,
                             "median_rounds": statistics.median(rounds),
                             "median_ms": statistics.median(ms)})
                if progress:
                    progress(f"{alg:8s} {topo:5s} n={n:5d} median rounds {rows[-1]['median_rounds']:9.1f} "
                             f"({conv}/{len(seeds)} converged)")
            table[alg][topo] = rows
    return table


def ordering_checks(table):
    """The report's qualitative claims, checked per node count on the seed medians.
    Returns {claim: {"holds": k, "of": m, "failing_n": [...]}}."""
    claims = {
        "full fastest": lambda m: m["full"] <= min(m.values()),
        "line slowest": lambda m: m["line"] >= max(m.values()),
        "Imp3D <= 3D": lambda m: m["Imp3D"] <= m["3D"],
    }
    out = {}
    for alg, per_topo in table.items():
        if not all(t in per_topo for t in TOPOLOGIES):
            continue
        ns = [row["n"] for row in per_topo["line"]]
        for name, pred in claims.items():
            fails = []
            for k, n in enumerate(ns):
                med = {t: per_topo[t][k]["median_rounds"] for t in TOPOLOGIES}
                if not pred(med):
                    fails.append(n)
            out[f"{alg}: {name}"] = {"holds": len(ns) - len(fails), "of": len(ns), "failing_n": fails}
    return out


def report_ordering_checks():
    """The same claims on the digitised Report.pdf values (markers present only)."""
    out = {}
    for alg, per_topo in REPORT_MS.items():
        for name in ("full fastest", "line slowest", "Imp3D <= 3D"):
            holds = of = 0
            for k in range(len(REPORT_NODES)):
                vals = {t: per_topo[t][k] for t in TOPOLOGIES}
                if name == "Imp3D <= 3D":
                    if vals["Imp3D"] is None or vals["3D"] is None:
                        continue
                    ok = vals["Imp3D"] <= vals["3D"]
                else:
                    if any(v is None for v in vals.values()):
                        continue
                    ok = vals["full"] <= min(vals.values()) if name == "full fastest" else \
                        vals["line"] >= max(vals.values())
                holds += int(ok)
                of += 1
            out[f"{alg}: {name}"] = {"holds": holds, "of": of}
    return out


def to_markdown(table, checks, ref_checks, seeds):
    lines = [f"# Report-curve sweep (median convergence rounds over seeds {list(seeds)})", ""]
    for alg, per_topo in table.items():
        ns = [row["n"] for row in next(iter(per_topo.values()))]
        lines.append(f"## {alg}")
        lines.append("")
        lines.append("| topology | " + " | ".join(str(n) for n in ns) + " |")
        lines.append("|---|" + "---|" * len(ns))
        for topo, rows in per_topo.items():
            cells = []
            for row in rows:
                c = f"{row['median_rounds']:g}"
                if row["converged"] < len(row["rounds"]):
                    c += f" ({row['converged']}/{len(row['rounds'])} conv)"
                cells.append(c)
            lines.append(f"| {topo} | " + " | ".join(cells) + " |")
        lines.append("")
        lines.append("median GPU wall ms: " + "; ".join(
            f"{topo} " + ", ".join(f"{row['median_ms']:.1f}" for row in rows) for topo, rows in per_topo.items()))
        lines.append("")
    lines.append("## Qualitative claims (this build: rounds; Report.pdf: digitised ms)")
    lines.append("")
    lines.append("| claim | this build | Report.pdf |")
    lines.append("|---|---|---|")
    for k, v in checks.items():
        r = ref_checks.get(k, {"holds": 0, "of": 0})
        fail = f" (fails at n={v['failing_n']})" if v["failing_n"] else ""
        lines.append(f"| {k} | {v['holds']}/{v['of']}{fail} | {r['holds']}/{r['of']} |")
    lines.append("")
    return "\n".join(lines)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=5)
    ap.add_argument("--nodes", default=",".join(str(n) for n in REPORT_NODES))
    ap.add_argument("--out", default="gpurun_out/report_curves")
    ap.add_argument("--max-rounds", type=int, default=10**6)
    a = ap.parse_args()
    nodes = [int(x) for x in a.nodes.split(",")]
    seeds = tuple(range(1, a.seeds + 1))
    t0 = time.time()
    table = sweep(product_runner(max_rounds=a.max_rounds), nodes=nodes, seeds=seeds,
                  progress=lambda s: print(s, flush=True))
    checks = ordering_checks(table)
    ref_checks = report_ordering_checks()
    os.makedirs(a.out, exist_ok=True)
    with open(os.path.join(a.out, "report_curves.json"), "w") as fh:
        json.dump({"seeds": list(seeds), "table": table, "checks": checks, "report_checks": ref_checks}, fh, indent=1)
    with open(os.path.join(a.out, "report_curves.md"), "w") as fh:
        fh.write(to_markdown(table, checks, ref_checks, seeds))
    print(json.dumps(checks, indent=1))
    print(f"sweep took {time.time() - t0:.1f} s", flush=True)


if __name__ == "__main__":
    main()
