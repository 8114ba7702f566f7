"""CPU, world_size 2 (and 3) over gloo: the multi-GPU decomposition of
libgossip_hip.so -- slab plan, halo refresh, slot-tagged random-edge messages,
rank-summed bookkeeping, replicated injector -- restated in numpy
(tests/multirank_emu.py) and run as real torch.distributed ranks; the gathered
result must equal the single-process CPU oracle bit for bit."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from tests.oracle_ctypes import Oracle


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, case, out_dir):
    import torch.distributed as dist
    from tests.multirank_emu import RankSim
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, topo, alg, seed, rounds = case
    sim = RankSim(n, topo, alg, seed, rank, world, dist)
    alerts = sim.step(rounds)
    lo, c, s, w, flags = sim.state()
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), lo=lo, alerts=np.array(alerts, dtype=np.int64),
             c=c if c is not None else np.zeros(0, np.int32), s=s if s is not None else np.zeros(0),
             w=w if w is not None else np.zeros(0), flags=flags, rounds=sim.round)
    dist.barrier()
    dist.destroy_process_group()


CASES = [  # (num_nodes, topology, algorithm, seed, rounds, world)
    (1728, "Imp3D", "push-sum", 5, 80, 2),
    (1000, "Imp3D", "gossip", 7, 400, 2),
    (1331, "3D", "push-sum", 9, 60, 2),
    (512, "3D", "gossip", 4, 300, 3),
    (300, "line", "gossip", 6, 1500, 2),
    (200, "line", "push-sum", 2, 200, 3),
    (2197, "Imp3D", "push-sum", 11, 50, 3),
    (3000, "full", "push-sum", 8, 200, 2),
    (2000, "full", "push-sum", 5, 150, 3),
    (1500, "full", "gossip", 3, 3000, 2),
    (999, "full", "gossip", 9, 3000, 3),
]


@pytest.mark.parametrize("n,topo,alg,seed,rounds,world", CASES, ids=lambda v: str(v))
def test_gloo_ranks_match_oracle(n, topo, alg, seed, rounds, world):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), (n, topo, alg, seed, rounds), d), nprocs=world, join=True)
        parts = [np.load(os.path.join(d, f"r{r}.npz")) for r in range(world)]
        orc = Oracle(n, topo, alg, seed)
        oa = orc.step(rounds)
        for p in parts:
            assert list(p["alerts"]) == oa, "per-round alerts differ from the oracle"
            assert int(p["rounds"]) == orc.rounds
        ref = orc.state()
        for p in parts:
            lo = int(p["lo"])
            m = len(p["flags"])
            np.testing.assert_array_equal(p["flags"], ref["flags"][lo:lo + m])
            if alg == "gossip":
                np.testing.assert_array_equal(p["c"], ref["c"][lo:lo + m])
            else:
                np.testing.assert_array_equal(p["s"], ref["s"][lo:lo + m])
                np.testing.assert_array_equal(p["w"], ref["w"][lo:lo + m])
        assert sum(len(p["flags"]) for p in parts) == orc.P
        orc.close()
