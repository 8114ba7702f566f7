"""Report-curve harness (tools/report_curves.py): the CPU oracle drives the sweep at
small sizes (ordering claims, table shape); on the GPU the product's sweep must
give the oracle's convergence rounds exactly."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import report_curves as rc  # noqa: E402

from .oracle_ctypes import Oracle


def oracle_runner(n, topology, algorithm, seed):
    o = Oracle(n, topology, algorithm, seed=seed, threads=1)
    try:
        o.run(max_rounds=10**6)
        return o.rounds, o.alerts_total >= o.T, 0.0
    finally:
        o.close()


def test_sweep_oracle_push_sum_ordering():
    table = rc.sweep(oracle_runner, nodes=(100, 300), seeds=(1, 2), algorithms=("push-sum",))
    assert set(table["push-sum"]) == set(rc.TOPOLOGIES)
    for rows in table["push-sum"].values():
        assert [r["n"] for r in rows] == [100, 300]
        assert all(r["converged"] == 2 for r in rows)
    checks = rc.ordering_checks(table)
    # README.md:3 / Report.pdf p.2: full fastest, line slowest
    assert checks["push-sum: full fastest"]["holds"] == 2
    assert checks["push-sum: line slowest"]["holds"] == 2
    md = rc.to_markdown(table, checks, rc.report_ordering_checks(), (1, 2))
    assert "| line |" in md and "push-sum: full fastest" in md


def test_report_digitised_checks():
    ref = rc.report_ordering_checks()
    # gossip plot: full is the lowest curve at every node count with all four markers
    assert ref["gossip: full fastest"]["holds"] == ref["gossip: full fastest"]["of"] > 0
    assert ref["push-sum: Imp3D <= 3D"]["of"] == 4


@pytest.mark.gpu
def test_sweep_product_matches_oracle():
    nodes, seeds = (100, 200), (1, 2)
    want = rc.sweep(oracle_runner, nodes=nodes, seeds=seeds)
    got = rc.sweep(rc.product_runner(), nodes=nodes, seeds=seeds)
    for alg in rc.ALGORITHMS:
        for topo in rc.TOPOLOGIES:
            assert [r["rounds"] for r in got[alg][topo]] == [r["rounds"] for r in want[alg][topo]], (alg, topo)
            assert [r["converged"] for r in got[alg][topo]] == [r["converged"] for r in want[alg][topo]]
