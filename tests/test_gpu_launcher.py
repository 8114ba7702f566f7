"""GPU: multi-GPU runs through the drop-in surface, rehearsed on one MI355X.

The reference's one entry point is `main` with positional argv, stopping at the
T-th alert (Program.fs:31-34,53-56).  `gossip ... --gpus G` (C++ CLI), `python -m
gossipprotocol_amd ... --gpus G` and `bench.py --gpus G` start one rank process
per GPU before anything touches a GPU (csrc/gossip_cli.cpp, gossipprotocol_amd/
launch.py); the ranks join through gp_rendezvous_id + gp_create_rank.  On the
one-GPU test box `--device 0` (CLI) / GP_BENCH_DEVICE=0 (bench) put every rank on
device 0 over RCCL's socket transport -- the same launch, rendezvous, slab plan
and exchange as on a multi-GPU node.  A multi-rank run must converge in exactly
the round a single-GPU run does (the convergence round is bit-exact for any rank
count), and its output must say how many GPUs it used.
"""
import json
import os
import re
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "gossipprotocol_amd", "gossip")


def _stats(out):
    m = re.search(r"rounds=(\d+) population=(\d+) threshold=(\d+) gpus=(\d+)", out)
    assert m, out
    return tuple(int(x) for x in m.groups())


@pytest.mark.parametrize("n,topo,alg", [(10**6, "Imp3D", "push-sum"), (27000, "Imp3D", "gossip"),
                                        (20000, "full", "push-sum"), (3000, "line", "gossip")])
def test_cli_gpus_matches_one_gpu(n, topo, alg):
    """`gossip n topo alg --gpus 2` converges in the same round as one GPU and keeps
    the stdout contract (Program.fs:198,203,55) on rank 0 only."""
    one = subprocess.run([EXE, str(n), topo, alg, "--stats"], capture_output=True, text=True, timeout=300)
    assert one.returncode == 0, one.stderr
    two = subprocess.run([EXE, str(n), topo, alg, "--gpus", "2", "--device", "0", "--stats"], capture_output=True,
                         text=True, timeout=300)
    assert two.returncode == 0, two.stderr[-3000:]
    lines = two.stdout.splitlines()
    assert lines[0] == ("Gossip Starts" if alg == "gossip" else "Push Sum Starts")
    assert lines[1].startswith("Convergence Time: ") and len(lines) == 3, two.stdout
    r1, p1, t1, g1 = _stats(one.stdout)
    r2, p2, t2, g2 = _stats(two.stdout)
    assert (g1, g2) == (1, 2)
    assert (r2, p2, t2) == (r1, p1, t1), "the two-rank run converged in a different round"


def test_cli_gossip_gpus_env():
    """GOSSIP_GPUS=3 is the same as --gpus 3."""
    env = dict(os.environ, GOSSIP_GPUS="3")
    one = subprocess.run([EXE, "64000", "Imp3D", "push-sum", "--stats"], capture_output=True, text=True, timeout=300,
                         env=dict(os.environ, GOSSIP_GPUS="1"))
    three = subprocess.run([EXE, "64000", "Imp3D", "push-sum", "--device", "0", "--stats"], capture_output=True,
                           text=True, timeout=300, env=env)
    assert one.returncode == 0 and three.returncode == 0, three.stderr[-3000:]
    assert _stats(three.stdout)[3] == 3 and _stats(three.stdout)[0] == _stats(one.stdout)[0]


def test_cli_gpus_beyond_visible_fails_loudly():
    """--gpus (visible + 1) without --device: the last rank has no device, so the
    launcher stops the others and fails -- it never runs on fewer GPUs than asked."""
    import torch  # device_count() does not initialise the GPU on this image
    n = max(1, torch.cuda.device_count())
    r = subprocess.run([EXE, "27000", "Imp3D", "push-sum", "--gpus", str(n + 1)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode != 0
    assert "Convergence Time" not in r.stdout
    assert f"rank {n}" in r.stderr


def test_python_cli_gpus_matches_one_gpu():
    def run(*extra):
        r = subprocess.run([sys.executable, "-m", "gossipprotocol_amd", "27000", "Imp3D", "push-sum", *extra],
                           capture_output=True, text=True, timeout=300, cwd=ROOT)
        assert r.returncode == 0, r.stderr[-3000:]
        return r.stdout.splitlines()
    one, two = run(), run("--gpus", "2", "--device", "0")
    assert two[0] == one[0] == "Push Sum Starts" and two[1].startswith("Convergence Time: ") and len(two) == 2


def test_bench_gpus_rehearsal_reports_world():
    """bench.py --gpus 2 without torch.distributed.run launches two ranks and says so."""
    env = dict(os.environ, GP_BENCH_DEVICE="0")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "10", "--warmup", "2", "--nodes",
                        str(200**3), "--no-cpu", "--no-traffic"], capture_output=True, text=True, timeout=400,
                       cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout  # one JSON line, nothing else on stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 10
    assert "rehearsal" in out["config"]["transport"] and out["config"]["launcher"].startswith("bench.py")
    assert out["config"]["population"] == 200**3 and out["value"] > 0
