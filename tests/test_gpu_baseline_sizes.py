"""GPU parity at BASELINE.json's sizes (C3, C4, C5 resolved).

The shipped default kernel of each configuration runs at the size the metric is
quoted on and is compared with the SRS v1 C oracle (oracle/srs_oracle.c) round
by round: per-round alert counts every round, the full node state at every
segment end.  Each configuration is one long run split into segments (one test
per segment, sharing the run through a module fixture) so the run reports
progress while it goes; a failing segment stops the run (-x).

  C3  gossip   Imp3D n = 1e8 (g = 465, P = 100,544,625): column-march kernel with
      runtime x-segments, 120 rounds (Program.fs:84-98,141-163 via SRS v1 B.3);
  C4  push-sum full  n = 1e8 (P = 100,000,001): through convergence
      (Program.fs:101-131,209-216 via SRS v1 B.4), every round's alerts and the
      full state every 30 rounds;
  C5  push-sum Imp3D n = 1e8 (g = 465): through activation (every node active)
      and then steady-state rounds, i.e. the headline kernel's all-active path
      (sender Philox redraw, compact in-edge messages) at the 1e8 scale.
      The 1e9 size itself is covered by tests/test_gpu_parity.py::
      test_full_size_1e9_* (one shared run, five segments): four checked rounds
      (activation, steady state, the alert peak at round 533, the converged tail
      at round 700)
      recomputed by the oracle for ~1.1e6 sampled receivers, bit-exact (a whole
      oracle run at 1e9 would need ~70 GB and ~20 min).
"""
import os
import sys

import numpy as np
import pytest

from tests.oracle_ctypes import Oracle

pytestmark = pytest.mark.gpu


class Pair:
    """The HIP simulation and the oracle advanced in lock step."""

    def __init__(self, n, topo, alg, seed):
        from gossipprotocol_amd import Simulation
        self.alg = alg
        self.sim = Simulation(n, topo, alg, seed=seed, kernel_timing=True)
        self.orc = Oracle(n, topo, alg, seed)
        assert (self.sim.population, self.sim.threshold, self.sim.seed_node) == \
            (self.orc.P, self.orc.T, self.orc.seed_node)
        self.finished = False

    def advance(self, k):
        ga = self.sim.step(k)
        oa = self.orc.step(k)
        assert ga == oa, f"per-round alerts differ in rounds {self.orc.rounds - len(oa)}..{self.orc.rounds}"
        if len(ga) < k:
            self.finished = True
        return ga

    def compare_state(self, chunk=25_000_000):
        P = self.orc.P
        for first in range(0, P, chunk):
            cnt = min(chunk, P - first)
            gs, os_ = self.sim.state(first, cnt), self.orc.state(first, cnt)
            if self.alg == "gossip":
                np.testing.assert_array_equal(gs["c"], os_["c"])
            else:
                np.testing.assert_array_equal(gs["s"], os_["s"])
                np.testing.assert_array_equal(gs["w"], os_["w"])
            np.testing.assert_array_equal(gs["flags"], os_["flags"])

    def close(self):
        self.sim.close()
        self.orc.close()


def progress(msg):
    print(f"[baseline-sizes] {msg}", file=sys.__stderr__, flush=True)


# ------------------------------------------------------------------ C3
@pytest.fixture(scope="module")
def c3():
    p = Pair(10**8, "Imp3D", "gossip", 1)
    yield p
    p.close()


def test_c3_default_kernel(c3):
    assert c3.sim.population == 100_544_625
    c3.advance(1)
    _, _, name = c3.sim.kernel_stats()
    assert "col" in name, f"C3 default kernel is {name}, expected the column march"


@pytest.mark.parametrize("seg", range(6))
def test_c3_gossip_imp3d_1e8(c3, seg):
    c3.advance(20)
    c3.compare_state()
    progress(f"C3 round {c3.orc.rounds}: alerts {c3.orc.alerts_total}")


# ------------------------------------------------------------------ C5 at 1e8
@pytest.fixture(scope="module")
def c5():
    p = Pair(10**8, "Imp3D", "push-sum", 1)
    yield p
    p.close()


@pytest.mark.parametrize("seg", range(12))
def test_c5_imp3d_pushsum_1e8_through_activation(c5, seg):
    if c5.orc.active_count() == c5.orc.P and getattr(c5, "steady", 0) >= 12:
        pytest.skip("activation done and 12 steady-state rounds compared")
    c5.advance(8)
    c5.compare_state()
    if c5.orc.active_count() == c5.orc.P:
        assert c5.sim.info().active == c5.sim.population
        c5.steady = getattr(c5, "steady", 0) + 8
    progress(f"C5@1e8 round {c5.orc.rounds}: active {c5.orc.active_count()}")


def test_c5_reached_steady_state(c5):
    assert c5.orc.active_count() == c5.orc.P, "activation did not complete within the compared rounds"
    assert getattr(c5, "steady", 0) >= 8, "fewer than 8 all-active rounds were compared"


# ------------------------------------------------------------------ C4
@pytest.fixture(scope="module")
def c4():
    p = Pair(10**8, "full", "push-sum", 1)
    yield p
    p.close()


@pytest.mark.parametrize("seg", range(25))
def test_c4_full_pushsum_1e8_to_convergence(c4, seg):
    """~550-600 rounds to convergence at P = 1e8 (oracle: 195 at 1e6, 385 at 1e7).
    The default suite compares the first 4 segments (activation, 120 rounds) state
    for state; the whole run is compared through convergence against the oracle's
    recorded run (test_run_to_convergence_matches_oracle_record).  GP_BASELINE_FULL=1
    runs the lock-step comparison through convergence (~5 min of oracle CPU)."""
    if c4.finished:
        pytest.skip("converged")
    if seg >= 4 and os.environ.get("GP_BASELINE_FULL") != "1":
        pytest.skip("lock-step past 120 rounds: GP_BASELINE_FULL=1 (the recorded oracle run covers convergence)")
    c4.advance(30)
    c4.compare_state()
    progress(f"C4 round {c4.orc.rounds}: alerts {c4.orc.alerts_total} of {c4.orc.T}")


def test_c4_converged(c4):
    if os.environ.get("GP_BASELINE_FULL") != "1":
        pytest.skip("lock-step to convergence: GP_BASELINE_FULL=1 (test_run_to_convergence_matches_oracle_record)")
    assert c4.finished and c4.sim.alerts_total >= c4.sim.threshold
    assert c4.sim.rounds == c4.orc.rounds


# ------------------------------------------------------------------ whole runs vs the oracle's record
GOLDEN_RUNS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "runs_1e8.json")


@pytest.mark.parametrize("case", ["c2", "c4", "c5_1e8"])
def test_run_to_convergence_matches_oracle_record(case):
    """The product run to convergence at a BASELINE size reproduces the C oracle's
    recorded run (tests/golden/make_golden_runs.py): every round's alert count
    (the scheduler's Alert stream, Program.fs:51-56), the convergence round, and an
    xxh3-128 digest of the whole final state (s, w, flags)."""
    import json
    from gossipprotocol_amd import Simulation
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "helpers"))
    from rccl_worker import slab_digest
    if not os.path.exists(GOLDEN_RUNS) or case not in json.load(open(GOLDEN_RUNS)):
        pytest.skip("no recorded oracle run")
    g = json.load(open(GOLDEN_RUNS))[case]
    with Simulation(g["num_nodes"], g["topology"], g["algorithm"], seed=g["seed"]) as sim:
        assert (sim.population, sim.threshold) == (g["population"], g["threshold"])
        alerts = []
        while sim.alerts_total < sim.threshold:
            a = sim.step(256)
            if not a:
                break
            alerts += a
            progress(f"{case} round {sim.rounds}: alerts {sim.alerts_total}")
        assert sim.rounds == g["rounds"]
        assert alerts == g["alerts_per_round"]
        assert slab_digest(sim, 0, sim.population) == g["final_state_xxh3_128"]

