"""GPU: the RCCL transport on the one GPU a test box has -- a one-rank RCCL
communicator (GP_FORCE_RCCL=1, experiments build) runs the split bookkeeping (pre / all-reduce /
post) and must match the single-rank path bit for bit.  Multi-rank RCCL runs
as separate processes: test_gpu_rccl_multiproc.py."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("topo,alg,n", [("Imp3D", "push-sum", 27000), ("Imp3D", "gossip", 27000),
                                        ("line", "gossip", 2000)])
def test_one_rank_rccl_matches_single(topo, alg, n, monkeypatch):
    import torch.distributed as dist
    from gossipprotocol_amd import Simulation
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29517")
    if not dist.is_initialized():
        dist.init_process_group("gloo", rank=0, world_size=1)
    monkeypatch.setenv("GP_FORCE_RCCL", "1")
    a = Simulation(n, topo, alg, seed=4, rank=0, world=1, dist=dist, experimental=True)
    monkeypatch.delenv("GP_FORCE_RCCL")
    b = Simulation(n, topo, alg, seed=4)
    assert a.step(400) == b.step(400)
    sa, sb = a.state(), b.state()
    for k in ("c", "s", "w", "flags"):
        np.testing.assert_array_equal(sa[k], sb[k])
    a.close()
    b.close()
