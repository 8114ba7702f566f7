"""CPU: the rank launchers and the rendezvous of the multi-GPU drop-in surface
(no GPU here, so every GPU call fails -- which is exactly what must not turn
into a silent one-GPU run).  The GPU side is tests/test_gpu_launcher.py."""
import ctypes as C
import os
import subprocess
import sys
import time

from gossipprotocol_amd import _lib as L
from gossipprotocol_amd.launch import run_ranks

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "gossipprotocol_amd", "gossip")


def test_run_ranks_environment(tmp_path):
    """Every rank gets RANK / WORLD_SIZE / MASTER_* / GOSSIP_RDV like torch.distributed.run would."""
    script = ("import os,sys; open(os.path.join(sys.argv[1], 'r'+os.environ['RANK']), 'w').write("
              "' '.join(os.environ[k] for k in ('RANK','LOCAL_RANK','WORLD_SIZE','MASTER_ADDR','GOSSIP_RDV','X')))")
    rc = run_ranks([sys.executable, "-c", script, str(tmp_path)], 3, env_for_rank=lambda r: {"X": f"x{r}"})
    assert rc == 0
    rows = [open(tmp_path / f"r{r}").read().split() for r in range(3)]
    for r, row in enumerate(rows):
        assert row[:4] == [str(r), str(r), "3", "127.0.0.1"] and row[5] == f"x{r}"
    assert len({row[4] for row in rows}) == 1 and not os.path.exists(os.path.dirname(rows[0][4]))


def test_run_ranks_first_failure_stops_the_others():
    t0 = time.perf_counter()
    script = "import os,sys,time; r=int(os.environ['RANK']); time.sleep(0.3) if r == 1 else None; " \
             "sys.exit(5) if r == 1 else time.sleep(120)"
    rc = run_ranks([sys.executable, "-c", script], 3)
    assert rc == 5 and time.perf_counter() - t0 < 60


def test_run_ranks_result_codes():
    """ok_codes are results (the CLI's 3 = not converged), not failures: rank 0's code is returned."""
    assert run_ranks([sys.executable, "-c", "import sys; sys.exit(3)"], 2, ok_codes=(0, 3)) == 3
    assert run_ranks([sys.executable, "-c", "pass"], 2) == 0


def test_rendezvous_reader(tmp_path):
    """Ranks > 0 read rank 0's 128-byte id; a missing file times out, a short one is refused."""
    lib = L.lib()
    path = tmp_path / "rccl_id"
    want = bytes(range(128))
    path.write_bytes(want)
    uid = C.create_string_buffer(128)
    assert lib.gp_rendezvous_id(1, str(path).encode(), 1000, uid) == 0 and uid.raw == want
    t0 = time.perf_counter()
    assert lib.gp_rendezvous_id(2, str(tmp_path / "absent").encode(), 50, uid) == -5
    assert time.perf_counter() - t0 < 5 and b"waited" in lib.gp_last_error()
    (tmp_path / "short").write_bytes(b"x" * 10)
    assert lib.gp_rendezvous_id(1, str(tmp_path / "short").encode(), 50, uid) == -1
    assert lib.gp_rendezvous_id(0, b"", 50, uid) == -1


def test_rendezvous_reader_waits_for_publisher(tmp_path):
    """The reader polls until rank 0 renames its id into place."""
    lib = L.lib()
    path = tmp_path / "rccl_id"
    code = (f"import time,os; time.sleep(0.4); open('{path}.tmp','wb').write(bytes(128*[7])); "
            f"os.rename('{path}.tmp', '{path}')")
    p = subprocess.Popen([sys.executable, "-c", code])
    uid = C.create_string_buffer(128)
    assert lib.gp_rendezvous_id(3, str(path).encode(), 20000, uid) == 0 and uid.raw == bytes(128 * [7])
    p.wait()


def test_cli_gpus_without_gpu_fails_loudly():
    """`gossip ... --gpus 2` on a host without a GPU: non-zero, no convergence line,
    the launcher names the failing rank; the rendezvous directory is removed."""
    before = {d for d in os.listdir("/tmp") if d.startswith("gossip_rdv_")}
    r = subprocess.run([EXE, "1000", "Imp3D", "push-sum", "--gpus", "2"], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, TMPDIR="/tmp"))
    assert r.returncode != 0 and "Convergence Time" not in r.stdout
    assert "rank" in r.stderr
    after = {d for d in os.listdir("/tmp") if d.startswith("gossip_rdv_")}
    assert after <= before


def test_cli_gpus_argument_checks():
    r = subprocess.run([EXE, "1000", "Imp3D", "push-sum", "--gpus", "0"], capture_output=True, text=True)
    assert r.returncode == 2 and "--gpus" in r.stderr
    r = subprocess.run([EXE, "1000", "Imp3D", "push_sum", "--gpus", "4"], capture_output=True, text=True)
    assert r.returncode == 2 and r.stdout.strip() == "option invalid"


def test_create_num_gpus_points_to_the_launcher():
    """gp_create(num_gpus > 1) without virtual ranks names the launcher instead of running one GPU."""
    lib = L.lib()
    cfg = L.GpConfig(num_nodes=1000, topology=L.GP_IMP3D, algorithm=L.GP_PUSHSUM, seed=1, num_gpus=8)
    h = C.c_void_p()
    assert lib.gp_create(C.byref(cfg), C.byref(h)) == -1
    assert b"--gpus 8" in lib.gp_last_error() and not h.value


def test_bench_world_mismatch_refused():
    """WORLD_SIZE set by a launcher but different from --gpus: refused, not re-interpreted."""
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--no-cpu", "--no-traffic"], cwd=ROOT,
                       capture_output=True, text=True, timeout=120, env=dict(os.environ, WORLD_SIZE="1"))
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_rendezvous_stale_file_and_nonce(tmp_path, monkeypatch):
    """A reused rendezvous path: rank 0 refuses to publish over a file already there,
    and with GOSSIP_RDV_NONCE set (the launchers set one per launch) a reader takes
    only a file carrying its nonce -- a stale id from a crashed run is never read."""
    lib = L.lib()
    path = tmp_path / "rccl_id"
    path.write_bytes(bytes(128) + b"old-launch")
    uid = C.create_string_buffer(128)
    assert lib.gp_rendezvous_id(0, str(path).encode(), 50, uid) == -5
    assert b"already exists" in lib.gp_last_error()
    monkeypatch.setenv("GOSSIP_RDV_NONCE", "this-launch")
    assert lib.gp_rendezvous_id(1, str(path).encode(), 100, uid) == -5
    assert b"nonce" in lib.gp_last_error()
    want = bytes(range(128))
    path.write_bytes(want + b"this-launch")
    assert lib.gp_rendezvous_id(1, str(path).encode(), 100, uid) == 0 and uid.raw == want


def test_python_cli_world_mismatch_refused():
    """python -m gossipprotocol_amd under an external launcher (WORLD_SIZE set) runs as that
    rank instead of launching again, and refuses a --gpus that disagrees with WORLD_SIZE."""
    r = subprocess.run([sys.executable, "-m", "gossipprotocol_amd", "1000", "Imp3D", "push-sum", "--gpus", "2"],
                       cwd=ROOT, capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, WORLD_SIZE="4", RANK="0"))
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr


def test_bench_roofline_bytes_follow_survey():
    """bench.py's roofline counts SURVEY.md §8(d)'s algorithmic bytes per node-round:
    B_ps = 34 + 4 [Imp3D] + 32 a + 8 a_x in steady state -- C5 ~71, C2 66, C4 74 B."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    c5 = bench.survey_bytes_per_node("Imp3D", "push-sum", 1000)
    assert abs(c5 - (34 + 4 + 32 + 8 / 7)) < 2e-3  # 1/7 random-link sends, end planes barely move it
    assert bench.survey_bytes_per_node("3D", "push-sum", 100) == 66.0
    assert bench.survey_bytes_per_node("full", "push-sum", 0) == 74.0
    assert bench.survey_bytes_per_node("Imp3D", "gossip", 465) is None
    # a lattice of edge 2: every node is on an end plane of all three axes (3 neighbours, 1/4)
    assert abs(bench.survey_bytes_per_node("Imp3D", "push-sum", 2) - (70 + 8 / 4)) < 1e-12
